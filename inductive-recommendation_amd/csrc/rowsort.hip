// rowsort.hip - fixed-order accumulation of rows with repeated indices (gfx950).
//
// The backward of the BPR gathers (rep[users], rep[n_users + pos / neg],
// model.py:4048-4049; the Embedding lookups of trainer.py:544-546) is an
// index_put with accumulate: dst[idx[i]] += src[i] with repeated idx.  Run on
// one CPU thread, torch walks i in increasing order (with several threads it
// adds atomically in no fixed order), so every destination row receives its
// terms in the order they appear in idx.  Float atomics on the GPU would make
// that order - and so the low bits of the sums - depend on scheduling.  Here the
// (row, position) pairs are sorted once, and one thread per distinct row and
// 4-float chunk adds that row's terms in increasing position: the sequential
// order, the same bits on every run.
//
//   igr_rowsort               keys = sort((idx[i] + off) << 32 | i)
//   igr_scatter_add_rows_f32  dst[row] += src[i], i in increasing order per row
//   igr_rowset_sum_f32        agg[k] = sum of a row's sources, slot[row] = k
//
// Sort: tiles of 1024 keys are sorted by a bitonic network held in registers
// (lane shuffles, LDS only across waves), then every key
// finds its final position as its rank in its own run plus the number of
// smaller keys in every other run (binary searches; all keys are distinct).
// More than 64 runs are first merged pairwise the same way.  Every loop has a
// fixed trip count: nothing waits on another workgroup.
#include <algorithm>

#include "common.h"
#include "segsum.h"

namespace igr {

constexpr int kSortTile = 1024;     // keys per LDS-sorted tile
constexpr int kSortThreads = 256;   // 4 keys per thread
constexpr int kMaxRankRuns = 64;    // runs ranked against each other in one pass
constexpr uint64_t kPadRow = 0xffffffffull;

__device__ __forceinline__ uint64_t make_key(int64_t n, const int64_t *__restrict__ i0, int64_t o0,
                                             const int64_t *__restrict__ i1, int64_t o1,
                                             const int64_t *__restrict__ i2, int64_t o2, int64_t total, int64_t e) {
    if (e >= total) return (kPadRow << 32) | (uint64_t)(uint32_t)e;  // pads: distinct, after every real key
    const int64_t a = e / n, i = e - a * n;
    const int64_t row = a == 0 ? i0[i] + o0 : (a == 1 ? i1[i] + o1 : i2[i] + o2);
    return ((uint64_t)row << 32) | (uint64_t)(uint32_t)e;
}

// keep the smaller (keep_min) or the larger of v and its partner's value
__device__ __forceinline__ uint64_t cmpx(uint64_t v, uint64_t pv, bool keep_min) {
    return ((v < pv) == keep_min) ? v : pv;
}

// Sort each tile of kSortTile keys (built on the fly from up to three index
// arrays).  Thread t holds keys 4t .. 4t+3 of the bitonic network in registers:
// strides 1, 2 are exchanges inside the thread, strides 4 .. 128 lane shuffles
// inside the wave, and only strides 256, 512 (three stages in all) cross waves
// through LDS - the network is latency-bound, and a shuffle costs a fraction of
// an LDS round trip plus barrier.
__global__ __launch_bounds__(kSortThreads) void rowsort_tiles_kernel(
    int64_t n, const int64_t *__restrict__ i0, int64_t o0, const int64_t *__restrict__ i1, int64_t o1,
    const int64_t *__restrict__ i2, int64_t o2, int64_t total, uint64_t *__restrict__ out) {
    __shared__ uint64_t s[kSortTile];
    const int tid = threadIdx.x;
    const int64_t base = (int64_t)blockIdx.x * kSortTile;
    uint64_t v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = make_key(n, i0, o0, i1, o1, i2, o2, total, base + tid * 4 + r);
#pragma unroll
    for (int k = 2; k <= kSortTile; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            if (j >= 256) {
#pragma unroll
                for (int r = 0; r < 4; ++r) s[tid * 4 + r] = v[r];
                __syncthreads();
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = tid * 4 + r;
                    v[r] = cmpx(v[r], s[i ^ j], ((i & j) == 0) == ((i & k) == 0));
                }
                __syncthreads();
            } else if (j >= 4) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = tid * 4 + r;
                    const uint64_t pv = (uint64_t)__shfl_xor((unsigned long long)v[r], j >> 2, 64);
                    v[r] = cmpx(v[r], pv, ((i & j) == 0) == ((i & k) == 0));
                }
            } else {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    if ((r & j) == 0) {
                        const bool up = ((tid * 4 + r) & k) == 0;
                        const uint64_t a = v[r], b = v[r | j];
                        if ((a > b) == up) {
                            v[r] = b;
                            v[r | j] = a;
                        }
                    }
                }
            }
        }
    }
    // 32-byte chunks per thread: two 16-byte stores
    ulonglong2 *o = reinterpret_cast<ulonglong2 *>(out + base + tid * 4);
    o[0] = make_ulonglong2(v[0], v[1]);
    o[1] = make_ulonglong2(v[2], v[3]);
}

// number of keys in the sorted run [run, run + len) that are smaller than key
__device__ __forceinline__ int64_t lower_bound_run(const uint64_t *__restrict__ run, int64_t len, uint64_t key) {
    int64_t lo = 0, hi = len;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (run[mid] < key) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// Pairwise merge of sorted runs of run_len keys: a key's position in the merged
// run is its rank in its own run plus its rank in the partner run.
__global__ void rowsort_merge_pairs_kernel(int64_t n_pad, int64_t run_len, const uint64_t *__restrict__ in,
                                           uint64_t *__restrict__ out) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n_pad) return;
    const int64_t run = p / run_len, pair = run >> 1;
    const int64_t partner = (run ^ 1) * run_len;
    const uint64_t key = in[p];
    const int64_t rank = (p - run * run_len) + lower_bound_run(in + partner, run_len, key);
    out[pair * 2 * run_len + rank] = key;
}

// Final pass: n_runs (<= kMaxRankRuns) sorted runs of run_len keys (a power of
// two) -> one sorted array.  A key's final position is its rank in its own run
// plus the number of smaller keys in every other run.  The searches are
// branch-free bisections with a fixed trip count, and a thread advances the
// searches of its four keys in up to eight runs together, step by step, so up
// to 32 independent probes are in flight instead of one dependent chain.
// LDS: the whole input is staged in LDS first (n_pad <= 8192 keys).
template <bool LDS>
__global__ __launch_bounds__(kSortThreads) void rowsort_rank_kernel(int64_t n_pad, int64_t run_len, int n_runs,
                                                                    const uint64_t *__restrict__ in,
                                                                    uint64_t *__restrict__ out) {
    __shared__ __align__(16) uint64_t s[LDS ? 8192 : 2];
    const uint64_t *src = in;
    if (LDS) {
        const ulonglong2 *in2 = reinterpret_cast<const ulonglong2 *>(in);
        for (int64_t t = threadIdx.x; t < n_pad / 2; t += kSortThreads) reinterpret_cast<ulonglong2 *>(s)[t] = in2[t];
        __syncthreads();
        src = s;
    }
    constexpr int RB = 8;  // runs searched together
    const int64_t p0 = (int64_t)blockIdx.x * kSortTile + threadIdx.x;  // keys p0 + r * kSortThreads, r < 4
    const int own = (int)(p0 / run_len);  // a tile lies inside one run
    uint64_t key[4];
    int64_t rank[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int64_t p = p0 + r * kSortThreads;
        key[r] = src[p];
        rank[r] = p - (int64_t)own * run_len;
    }
    for (int rb = 0; rb < n_runs; rb += RB) {
        int64_t pos[4][RB];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int u = 0; u < RB; ++u) pos[r][u] = 0;
        // pos = number of keys < key among the run's first run_len - 1 keys ...
        for (int64_t step = run_len >> 1; step >= 1; step >>= 1) {
#pragma unroll
            for (int u = 0; u < RB; ++u) {
                const int run = rb + u;
                if (run < n_runs && run != own) {
                    const uint64_t *base = src + (int64_t)run * run_len;
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        if (base[pos[r][u] + step - 1] < key[r]) pos[r][u] += step;
                }
            }
        }
#pragma unroll
        for (int u = 0; u < RB; ++u) {
            const int run = rb + u;
            if (run < n_runs && run != own) {
                const uint64_t *base = src + (int64_t)run * run_len;
#pragma unroll
                for (int r = 0; r < 4; ++r)  // ... and the last one
                    rank[r] += pos[r][u] + (base[pos[r][u]] < key[r] ? 1 : 0);
            }
        }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) out[rank[r]] = key[r];
}

static int64_t pow2_ceil(int64_t v) {
    int64_t p = 1;
    while (p < v) p <<= 1;
    return p;
}

// padded key count of a sort of `total` keys
static int64_t sort_pad(int64_t total) {
    const int64_t tiles = (total + kSortTile - 1) / kSortTile;
    return kSortTile * (tiles <= kMaxRankRuns ? std::max<int64_t>(tiles, 1) : pow2_ceil(tiles));
}

}  // namespace igr

using namespace igr;

extern "C" int64_t igr_rowsort_size(int64_t total) { return total <= 0 ? 0 : 2 * sort_pad(total); }

extern "C" int igr_rowsort(int64_t n, const int64_t *idx0, int64_t off0, const int64_t *idx1, int64_t off1,
                           const int64_t *idx2, int64_t off2, uint64_t *keys, void *stream) {
    return guarded("igr_rowsort", [&]() -> int {
        const char *fn = "igr_rowsort";
        if (n <= 0) return IGR_OK;
        if (!idx0 || !keys) return arg_error(fn, "idx0 / keys NULL");
        if (idx2 && !idx1) return arg_error(fn, "idx2 without idx1");
        const int64_t total = n * (idx2 ? 3 : (idx1 ? 2 : 1));
        if (total > 2147483647) return arg_error(fn, "more than 2^31 - 1 indices");
        const int64_t n_pad = sort_pad(total);
        const int64_t tiles = n_pad / kSortTile;
        hipStream_t st = reinterpret_cast<hipStream_t>(stream);
        // passes after the tile sort: pairwise merges down to <= kMaxRankRuns runs, then
        // one ranking pass (none for a single tile); ping-pong so the result lands in keys
        int merges = 0;
        for (int64_t r = tiles; r > kMaxRankRuns; r >>= 1) ++merges;
        const int passes = merges + (tiles > 1 ? 1 : 0);
        uint64_t *buf[2] = {keys, keys + n_pad};
        int cur = passes & 1;  // the tile sort writes here
        hipLaunchKernelGGL(rowsort_tiles_kernel, dim3((unsigned)tiles), dim3(kSortThreads), 0, st, n, idx0, off0,
                           idx1, off1, idx2, off2, total, buf[cur]);
        int64_t run_len = kSortTile, runs = tiles;
        for (int m = 0; m < merges; ++m) {
            hipLaunchKernelGGL(rowsort_merge_pairs_kernel, dim3((unsigned)((n_pad + 255) / 256)), dim3(256), 0, st,
                               n_pad, run_len, buf[cur], buf[cur ^ 1]);
            cur ^= 1;
            run_len <<= 1;
            runs >>= 1;
        }
        if (runs > 1) {
            if (n_pad <= 8192)
                hipLaunchKernelGGL((rowsort_rank_kernel<true>), dim3((unsigned)tiles), dim3(kSortThreads), 0, st, n_pad,
                                   run_len, (int)runs, buf[cur], buf[cur ^ 1]);
            else
                hipLaunchKernelGGL((rowsort_rank_kernel<false>), dim3((unsigned)tiles), dim3(kSortThreads), 0, st,
                                   n_pad, run_len, (int)runs, buf[cur], buf[cur ^ 1]);
            cur ^= 1;
        }
        if (cur != 0) return arg_error(fn, "internal: result not in keys");
        return launch_status(fn);
    });
}

extern "C" int igr_scatter_add_rows_f32(int64_t n, int32_t d, const uint64_t *sorted, const float *src,
                                        int64_t ld_src, float *dst, int64_t ld_dst, void *stream) {
    return guarded("igr_scatter_add_rows_f32", [&]() -> int {
        const char *fn = "igr_scatter_add_rows_f32";
        if (d <= 0 || ld_src < d || ld_dst < d) return arg_error(fn, "bad d / ld");
        if (n <= 0) return IGR_OK;
        if (!sorted || !src || !dst) return arg_error(fn, "sorted / src / dst NULL");
        if (n > 2147483647) return arg_error(fn, "too many rows");
        hipStream_t st = reinterpret_cast<hipStream_t>(stream);
        const bool vec = d % 4 == 0 && ld_src % 4 == 0 && ld_dst % 4 == 0 && aligned16(src) && aligned16(dst);
        const int64_t threads = n * (vec ? d / 4 : d);
        const dim3 grid((unsigned)((threads + 255) / 256));
        if (vec)
            hipLaunchKernelGGL((seg_scatter_add_kernel<SegAdd4>), grid, dim3(256), 0, st, n, (int)d / 4, sorted, src,
                               ld_src, dst, ld_dst);
        else
            hipLaunchKernelGGL((seg_scatter_add_kernel<SegAdd1>), grid, dim3(256), 0, st, n, (int)d, sorted, src,
                               ld_src, dst, ld_dst);
        return launch_status(fn);
    });
}

extern "C" int igr_rowset_sum_f32(int64_t n_sel, int32_t d, const uint64_t *sorted, const float *src, int64_t lds,
                                  float scale, int32_t *slot, float *agg, int64_t ld_agg, void *stream) {
    return guarded("igr_rowset_sum_f32", [&]() -> int {
        const char *fn = "igr_rowset_sum_f32";
        if (d <= 0 || lds < d || ld_agg < d) return arg_error(fn, "bad d / leading dims");
        if (n_sel <= 0) return IGR_OK;
        if (!sorted || !src || !slot || !agg) return arg_error(fn, "NULL pointer");
        if (n_sel > 2147483647) return arg_error(fn, "too many rows");
        hipStream_t st = reinterpret_cast<hipStream_t>(stream);
        const bool vec = d % 4 == 0 && lds % 4 == 0 && ld_agg % 4 == 0 && aligned16(src) && aligned16(agg);
        const int64_t threads = n_sel * (vec ? d / 4 : d);
        const dim3 grid((unsigned)((threads + 255) / 256));
        if (vec)
            hipLaunchKernelGGL((seg_rowset_sum_kernel<SegAdd4>), grid, dim3(256), 0, st, n_sel, (int)d / 4, sorted, src,
                               lds, scale, slot, agg, ld_agg);
        else
            hipLaunchKernelGGL((seg_rowset_sum_kernel<SegAdd1>), grid, dim3(256), 0, st, n_sel, (int)d, sorted, src,
                               lds, scale, slot, agg, ld_agg);
        return launch_status(fn);
    });
}
