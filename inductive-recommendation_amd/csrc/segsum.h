// segsum.h - fixed-order sums over runs of equal rows in a sorted key array
// (device templates shared by rowsort.hip and bpr.hip).
//
// keys[k] = (row << 32) | entry, ascending (igr_rowsort).  One thread per
// (position k, chunk f of the feature row); the thread at the first position of
// a row's run owns that row: it finds the run's end, then adds the run's source
// rows in key order, four loads in flight at a time (the adds stay in order).
#pragma once

#include "common.h"

namespace igr {

struct SegAdd4 {
    typedef float4 T;
    static __device__ __forceinline__ T zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }
    static __device__ __forceinline__ T load(const float *p, int f) { return reinterpret_cast<const float4 *>(p)[f]; }
    static __device__ __forceinline__ void store(float *p, int f, T v) { reinterpret_cast<float4 *>(p)[f] = v; }
    static __device__ __forceinline__ T fma(float s, T x, T a) { return f4_fma(s, x, a); }
    static __device__ __forceinline__ T add(T a, T x) { return f4_add(a, x); }
};
struct SegAdd1 {
    typedef float T;
    static __device__ __forceinline__ T zero() { return 0.f; }
    static __device__ __forceinline__ T load(const float *p, int f) { return p[f]; }
    static __device__ __forceinline__ void store(float *p, int f, T v) { p[f] = v; }
    static __device__ __forceinline__ T fma(float s, T x, T a) { return fmaf(s, x, a); }
    static __device__ __forceinline__ T add(T a, T x) { return a + x; }
};

// acc (+)= sum over the run of keys starting at k of [scale *] src[entry]; returns the sum.
// SCALED: acc = fma(scale, x, acc) per term; otherwise acc = acc + x.
template <class V, bool SCALED>
__device__ __forceinline__ typename V::T seg_run_sum(typename V::T acc, int64_t n, int64_t k, uint64_t row,
                                                     const uint64_t *__restrict__ keys,
                                                     const float *__restrict__ src, int64_t ld_src, int f,
                                                     float scale) {
    int64_t end = k + 1;
    while (end < n && (keys[end] >> 32) == row) ++end;
    int64_t q = k;
    for (; q + 4 <= end; q += 4) {
        const uint32_t e0 = (uint32_t)keys[q], e1 = (uint32_t)keys[q + 1], e2 = (uint32_t)keys[q + 2],
                       e3 = (uint32_t)keys[q + 3];
        const typename V::T x0 = V::load(src + (int64_t)e0 * ld_src, f), x1 = V::load(src + (int64_t)e1 * ld_src, f),
                            x2 = V::load(src + (int64_t)e2 * ld_src, f), x3 = V::load(src + (int64_t)e3 * ld_src, f);
        if (SCALED) {
            acc = V::fma(scale, x0, acc);
            acc = V::fma(scale, x1, acc);
            acc = V::fma(scale, x2, acc);
            acc = V::fma(scale, x3, acc);
        } else {
            acc = V::add(acc, x0);
            acc = V::add(acc, x1);
            acc = V::add(acc, x2);
            acc = V::add(acc, x3);
        }
    }
    for (; q < end; ++q) {
        const typename V::T x = V::load(src + (int64_t)(uint32_t)keys[q] * ld_src, f);
        acc = SCALED ? V::fma(scale, x, acc) : V::add(acc, x);
    }
    return acc;
}

// dst[row] += sum of the row's sources, in key order, onto the value dst holds
template <class V>
__global__ void seg_scatter_add_kernel(int64_t n, int per, const uint64_t *__restrict__ keys,
                                       const float *__restrict__ src, int64_t ld_src, float *__restrict__ dst,
                                       int64_t ld_dst) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * per) return;
    const int64_t k = t / per;
    const int f = (int)(t - k * per);
    const uint64_t row = keys[k] >> 32;
    if (k > 0 && (keys[k - 1] >> 32) == row) return;
    float *o = dst + (int64_t)row * ld_dst;
    V::store(o, f, seg_run_sum<V, false>(V::load(o, f), n, k, row, keys, src, ld_src, f, 1.f));
}

// agg[k] = sum of scale * the row's sources, slot[row] = k, at the first position k of every row
template <class V>
__global__ void seg_rowset_sum_kernel(int64_t n, int per, const uint64_t *__restrict__ keys,
                                      const float *__restrict__ src, int64_t ld_src, float scale,
                                      int32_t *__restrict__ slot, float *__restrict__ agg, int64_t ld_agg) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * per) return;
    const int64_t k = t / per;
    const int f = (int)(t - k * per);
    const uint64_t row = keys[k] >> 32;
    if (k > 0 && (keys[k - 1] >> 32) == row) return;
    if (f == 0) slot[row] = (int32_t)k;
    V::store(agg + k * ld_agg, f, seg_run_sum<V, true>(V::zero(), n, k, row, keys, src, ld_src, f, scale));
}

}  // namespace igr
