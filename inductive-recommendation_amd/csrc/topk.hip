// topk.hip - the eval ranking: train-item mask + per-user top-k of the score rows.
//
// BasicTrainer.eval (trainer.py:146-182): scores = rep[users] . rep[items]^T
// (igr_gemm_f32), scores[u, train items of u] = -inf, then topk(k = max topks)
// per user.  Here:
//   igr_mask_scores_f32: scores[r, cols[p]] = -inf for p in [row_ptr[r], row_ptr[r+1])
//   igr_topk_f32:        per row the k largest scores, sorted (value desc, index asc)
// One workgroup per row (topk_kernel below): a 12-bit histogram pass finds the
// bin holding the k-th largest order-preserving key, a second pass collects the
// keys above it and the bin's own elements into LDS, and the rest of the
// selection (ties broken by the smallest index, so the result is
// deterministic) runs in LDS; a bitonic sort orders the k (key, index) pairs.
// Measured on MI355X (scripts/bench_eval.py, Gowalla shape, 29,858 x 40,981
// scores): 8.6 ms with four 8-bit radix passes over memory, 3.2 ms this way;
// holding the row in registers and bounding the k-th value by the threads'
// slice maxima (one read of the row) took 4.7 ms - the LDS select phases, not
// the bytes, bound a row.
#include "common.h"

namespace igr {

constexpr int kTopkThreads = 1024;  // one workgroup (16 waves) per row
constexpr int kTopkMax = 1024;      // k <= kTopkMax (LDS sort buffer)
constexpr int kTopkBins = 4096;     // first digit: the key's top 12 bits (sign, exponent, 3 mantissa bits)
constexpr int kTopkCand = 4096;     // LDS capacity for the elements of the k-th value's bin

// -0.0 and +0.0 compare equal (as in torch / numpy): f + 0.0f maps -0.0 to +0.0
__device__ __forceinline__ uint32_t order_key(float f) {
    const uint32_t u = __float_as_uint(f + 0.0f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// Visit (j, key) for every element of a row: float4 loads when the row is
// 16-B aligned, scalar loads otherwise.
template <class F>
__device__ __forceinline__ void for_each_key(const float *row, int64_t n, F &&fn) {
    if ((reinterpret_cast<uintptr_t>(row) & 15u) == 0) {
        const int64_t n4 = n >> 2;
        const float4 *r4 = reinterpret_cast<const float4 *>(row);
        for (int64_t q = threadIdx.x; q < n4; q += kTopkThreads) {
            const float4 v = r4[q];
            fn(4 * q, order_key(v.x));
            fn(4 * q + 1, order_key(v.y));
            fn(4 * q + 2, order_key(v.z));
            fn(4 * q + 3, order_key(v.w));
        }
        for (int64_t j = 4 * n4 + threadIdx.x; j < n; j += kTopkThreads) fn(j, order_key(row[j]));
    } else {
        for (int64_t j = threadIdx.x; j < n; j += kTopkThreads) fn(j, order_key(row[j]));
    }
}

// Radix select: among elements j < n with pred(j) true, the `need`-th largest
// of kfn(j), 8 bits per pass.  Returns the key and sets *left = how many
// elements equal to it are still needed (1 .. need).  hist: >= 256 LDS ints.
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
        if (threadIdx.x < kWave) {  // one wave scans the 256 bins from the top
            const int lane = threadIdx.x;
            int c[4], tot = 0;
            for (int q = 0; q < 4; ++q) tot += (c[q] = hist[255 - 4 * lane - q]);
            int incl = tot;
            for (int o = 1; o < kWave; o <<= 1) {
                const int v = __shfl_up(incl, o, kWave);
                if (lane >= o) incl += v;
            }
            int acc = incl - tot;  // elements in higher bins than this lane's four
            if (acc < need && acc + tot >= need) {
                for (int q = 0; q < 4; ++q) {
                    if (acc + c[q] >= need) {
                        sh[0] = 255 - 4 * lane - q;
                        sh[1] = need - acc;
                        break;
                    }
                    acc += c[q];
                }
            }
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

// Among n keyed elements, those ranking in the top `need` (key descending,
// index ascending): returns the threshold key T, and TI / all_ties such that
// element (key, j) is selected iff key > T || (key == T && (all_ties || ~j >= TI)).
template <class KeyFn, class IdxFn>
__device__ void select_threshold(int64_t n, KeyFn kfn, IdxFn ifn, int need, int *hist, int *sh, uint32_t *T_out,
                                 uint32_t *TI_out, bool *all_ties_out) {
    int left;
    const uint32_t T = radix_select(n, kfn, [](int64_t) { return true; }, need, hist, sh, &left);
    if (threadIdx.x == 0) sh[2] = 0;
    __syncthreads();
    int cnt = 0;
    for (int64_t j = threadIdx.x; j < n; j += kTopkThreads) cnt += (kfn(j) == T);
    if (cnt) atomicAdd(&sh[2], cnt);
    __syncthreads();
    const int ties = sh[2];
    __syncthreads();
    bool all_ties = true;
    uint32_t TI = 0u;
    if (ties > left) {  // among the ties, the `left` smallest indices (largest ~index)
        all_ties = false;
        int dummy;
        TI = radix_select(
            n, [&](int64_t j) { return ~ifn(j); }, [&](int64_t j) { return kfn(j) == T; }, left, hist, sh, &dummy);
    }
    *T_out = T;
    *TI_out = TI;
    *all_ties_out = all_ties;
}

// Wave-aggregated append to an LDS list: returns the slot of this lane's item.
__device__ __forceinline__ int wave_append(bool take, int *counter) {
    const uint64_t mask = __ballot(take);
    if (!mask) return -1;
    const int lane = threadIdx.x & (kWave - 1);
    const int leader = __ffsll((unsigned long long)mask) - 1;
    int base = 0;
    if (lane == leader) base = atomicAdd(counter, __popcll(mask));
    base = __shfl(base, leader, kWave);
    return take ? base + __popcll(mask & ((1ull << lane) - 1ull)) : -1;
}

// One workgroup per row.  Pass 1: a 4096-bin histogram of the key's top 12
// bits, scanned from the top to find the bin B holding the k-th largest key.
// Pass 2: keys above B go straight to the result list (fewer than k), keys in
// B to an LDS candidate list; the remaining `need` are chosen among the
// candidates by an 8-bit radix select in LDS (ties: smallest indices).  Two
// reads of the row.  When B holds more than kTopkCand elements (heavy ties,
// e.g. an all -inf row), the row is selected by radix passes over global
// memory instead.  A bitonic sort then orders the k (key desc, index asc).
__global__ __launch_bounds__(kTopkThreads) void topk_kernel(int64_t n_rows, int64_t n_cols,
                                                            const float *__restrict__ scores, int64_t ld, int k,
                                                            float *__restrict__ out_val, int64_t *__restrict__ out_idx) {
    __shared__ int hist[kTopkBins];
    __shared__ int sh[8];
    __shared__ int wsum[kTopkThreads / kWave];
    __shared__ uint32_t ckey[kTopkCand];
    __shared__ int32_t cidx[kTopkCand];
    __shared__ uint32_t skey[kTopkMax];
    __shared__ int32_t sidx[kTopkMax];
    const int64_t r = blockIdx.x;
    if (r >= n_rows) return;
    const float *row = scores + r * ld;
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;

    for (int b = tid; b < kTopkBins; b += kTopkThreads) hist[b] = 0;
    if (tid < 8) sh[tid] = 0;
    __syncthreads();
    for_each_key(row, n_cols, [&](int64_t, uint32_t key) { atomicAdd(&hist[key >> 20], 1); });
    __syncthreads();
    // block scan of the bins from the top: thread t owns bins 4095-4t .. 4092-4t
    {
        int c[4], tot = 0;
        for (int q = 0; q < 4; ++q) tot += (c[q] = hist[kTopkBins - 1 - 4 * tid - q]);
        int incl = tot;
        for (int o = 1; o < kWave; o <<= 1) {
            const int v = __shfl_up(incl, o, kWave);
            if (lane >= o) incl += v;
        }
        if (lane == kWave - 1) wsum[wid] = incl;
        __syncthreads();
        int wbase = 0;
        for (int w = 0; w < wid; ++w) wbase += wsum[w];
        int acc = wbase + incl - tot;
        if (acc < k && acc + tot >= k) {
            for (int q = 0; q < 4; ++q) {
                if (acc + c[q] >= k) {
                    sh[0] = kTopkBins - 1 - 4 * tid - q;  // the bin B
                    sh[1] = acc;                           // elements above B (< k)
                    sh[2] = c[q];                          // elements in B
                    break;
                }
                acc += c[q];
            }
        }
    }
    __syncthreads();
    const uint32_t B = (uint32_t)sh[0];
    const int above = sh[1], in_bin = sh[2];
    __syncthreads();
    if (in_bin <= kTopkCand) {
        // pass 2: above B -> result list, in B -> candidates (sh[3], sh[4] are the counters)
        for_each_key(row, n_cols, [&](int64_t j, uint32_t key) {
            const uint32_t bin = key >> 20;
            const int s = wave_append(bin > B, &sh[3]);
            if (s >= 0) {
                skey[s] = key;
                sidx[s] = (int32_t)j;
            }
            const int c = wave_append(bin == B, &sh[4]);
            if (c >= 0) {
                ckey[c] = key;
                cidx[c] = (int32_t)j;
            }
        });
        __syncthreads();
        uint32_t T, TI;
        bool all_ties;
        select_threshold(
            in_bin, [&](int64_t j) { return ckey[j]; }, [&](int64_t j) { return (uint32_t)cidx[j]; }, k - above, hist,
            sh + 5, &T, &TI, &all_ties);
        if (tid == 0) sh[3] = above;
        __syncthreads();
        for (int j = tid; j < in_bin; j += kTopkThreads) {
            const uint32_t key = ckey[j];
            const int32_t ix = cidx[j];
            if (key > T || (key == T && (all_ties || ~(uint32_t)ix >= TI))) {
                const int s = atomicAdd(&sh[3], 1);
                skey[s] = key;
                sidx[s] = ix;
            }
        }
    } else {
        uint32_t T, TI;
        bool all_ties;
        auto vkey = [&](int64_t j) { return order_key(row[j]); };
        select_threshold(
            n_cols, vkey, [](int64_t j) { return (uint32_t)j; }, k, hist, sh + 5, &T, &TI, &all_ties);
        if (tid == 0) sh[3] = 0;
        __syncthreads();
        for_each_key(row, n_cols, [&](int64_t j, uint32_t key) {
            const bool take = key > T || (key == T && (all_ties || ~(uint32_t)j >= TI));
            const int s = wave_append(take, &sh[3]);
            if (s >= 0) {
                skey[s] = key;
                sidx[s] = (int32_t)j;
            }
        });
    }
    __syncthreads();
    int m = 1;
    while (m < k) m <<= 1;
    for (int s = k + tid; s < m; s += kTopkThreads) {  // pad: sorts after every real element
        skey[s] = 0u;
        sidx[s] = 0x7fffffff;
    }
    __syncthreads();
    // bitonic sort, descending by key, ascending by index among equal keys
    for (int size = 2; size <= m; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int t = tid; t < m / 2; t += kTopkThreads) {
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
    for (int s = tid; s < k; s += kTopkThreads) {
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
