// graph_host.cpp - host (CPU) graph construction for the igr library.
//
// Replaces the reference's Python/scipy construction, which is O(E) Python
// at model.py:4162-4170 and single-threaded scipy at utils.py:42-50 /
// model.py:89-98: hours at 200 M edges.  Here: multi-threaded counting sort
// by row + per-row sort by column, duplicate merge, transposed CSR, and the
// degree-binned row schedule consumed by the SpMM kernels.
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <string>
#include <numeric>
#include <thread>
#include <vector>

#include "common.h"

namespace igr {

// n_threads <= 0: IGR_NUM_THREADS, else OMP_NUM_THREADS, else min(hardware, 16).
static int resolve_threads(int32_t n_threads) {
    if (n_threads > 0) return n_threads;
    for (const char *v : {"IGR_NUM_THREADS", "OMP_NUM_THREADS"}) {
        const char *s = std::getenv(v);
        if (s && std::atoi(s) > 0) return std::atoi(s);
    }
    unsigned h = std::thread::hardware_concurrency();
    return h ? (int)std::min(h, 16u) : 4;
}

template <class F>
static void parallel_for(int64_t n, int nt, F &&fn) {
    if (n <= 0) return;
    if (nt <= 1 || n < 4096) {
        fn(0, n);
        return;
    }
    std::vector<std::thread> ts;
    const int64_t step = (n + nt - 1) / nt;
    for (int t = 0; t < nt; ++t) {
        const int64_t b = t * step, e = std::min(n, b + step);
        if (b >= e) break;
        ts.emplace_back([&fn, b, e]() { fn(b, e); });
    }
    for (auto &t : ts) t.join();
}

// fn(t) for t in [0, nt), one thread each (the caller's thread takes t = 0).
template <class F>
static void per_thread(int nt, F &&fn) {
    std::vector<std::thread> ts;
    for (int t = 1; t < nt; ++t) ts.emplace_back([&fn, t]() { fn(t); });
    fn(0);
    for (auto &t : ts) t.join();
}

// Exclusive prefix sum of counts[0..n) into ptr[0..n].
static void prefix(const int64_t *counts, int64_t n, int64_t *ptr) {
    ptr[0] = 0;
    for (int64_t i = 0; i < n; ++i) ptr[i + 1] = ptr[i] + counts[i];
}

}  // namespace igr

using namespace igr;

extern "C" int igr_csr_from_coo(int64_t n_rows, int64_t n_cols, int64_t nnz, const int64_t *row,
                                const int64_t *col, const float *val, int32_t dedup,
                                int64_t *row_ptr, int32_t *col_idx, float *val_out,
                                int64_t *edge_id, int64_t *nnz_out, int32_t n_threads) {
    return guarded("igr_csr_from_coo", [&]() -> int {
        const char *fn = "igr_csr_from_coo";
        if (n_rows < 0 || n_cols < 0 || nnz < 0) return arg_error(fn, "negative size");
        if (n_cols > INT32_MAX) return arg_error(fn, "n_cols exceeds int32 column index");
        if (!row_ptr || !nnz_out || (nnz > 0 && (!row || !col || !col_idx)))
            return arg_error(fn, "NULL array");
        const int nt = resolve_threads(n_threads);
        // validate indices
        std::atomic<int64_t> bad{-1};
        parallel_for(nnz, nt, [&](int64_t b, int64_t e) {
            for (int64_t i = b; i < e; ++i)
                if (row[i] < 0 || row[i] >= n_rows || col[i] < 0 || col[i] >= n_cols) {
                    bad.store(i);
                    return;
                }
        });
        if (bad.load() >= 0) return arg_error(fn, "index out of range at edge " + std::to_string(bad.load()));

        // 1. count per row (relaxed atomics), 2. row offsets
        std::vector<int64_t> cnt(n_rows, 0);
        parallel_for(nnz, nt, [&](int64_t b, int64_t e) {
            for (int64_t i = b; i < e; ++i) __atomic_fetch_add(&cnt[row[i]], 1, __ATOMIC_RELAXED);
        });
        std::vector<int64_t> off(n_rows + 1);
        prefix(cnt.data(), n_rows, off.data());
        // 3. scatter into row buckets (order inside a bucket is arbitrary) a key
        //    that sorts as (col, input position): (col << 32 | position) when both
        //    fit, so step 4 sorts plain integers in place (no indirect col[] lookups
        //    per comparison); the position alone otherwise
        const bool packed = nnz <= (int64_t)UINT32_MAX;
        std::vector<uint64_t> key(nnz);
        std::vector<int64_t> cur(off.begin(), off.end() - 1);
        parallel_for(nnz, nt, [&](int64_t b, int64_t e) {
            for (int64_t i = b; i < e; ++i)
                key[__atomic_fetch_add(&cur[row[i]], 1, __ATOMIC_RELAXED)] =
                    packed ? ((uint64_t)col[i] << 32) | (uint64_t)i : (uint64_t)i;
        });
        auto pos_of = [&](uint64_t k) -> int64_t { return packed ? (int64_t)(k & 0xffffffffu) : (int64_t)k; };
        // 4. sort each bucket by (col, input position) == stable sort by (row, col);
        //    count the entries each row keeps
        std::vector<int64_t> kept(n_rows, 0);
        parallel_for(n_rows, nt, [&](int64_t b, int64_t e) {
            for (int64_t r = b; r < e; ++r) {
                uint64_t *p0 = key.data() + off[r], *p1 = key.data() + off[r + 1];
                if (packed)
                    std::sort(p0, p1);
                else
                    std::sort(p0, p1, [&](uint64_t x, uint64_t y) {
                        return col[x] < col[y] || (col[x] == col[y] && x < y);
                    });
                int64_t k = 0;
                for (uint64_t *q = p0; q < p1; ++q)
                    if (!dedup || q == p0 || col[pos_of(*q)] != col[pos_of(*(q - 1))]) ++k;
                kept[r] = k;
            }
        });
        prefix(kept.data(), n_rows, row_ptr);
        // 5. write, summing duplicates in input order
        parallel_for(n_rows, nt, [&](int64_t b, int64_t e) {
            for (int64_t r = b; r < e; ++r) {
                int64_t o = row_ptr[r] - 1;
                for (int64_t q = off[r]; q < off[r + 1]; ++q) {
                    const int64_t i = pos_of(key[q]);
                    const float v = val ? val[i] : 1.f;
                    if (dedup && q > off[r] && col[i] == col[pos_of(key[q - 1])]) {
                        if (val_out) val_out[o] += v;
                    } else {
                        ++o;
                        col_idx[o] = (int32_t)col[i];
                        if (val_out) val_out[o] = v;
                        if (edge_id) edge_id[o] = i;
                    }
                }
            }
        });
        *nnz_out = row_ptr[n_rows];
        return IGR_OK;
    });
}

extern "C" int igr_count_ids(int64_t n, const int64_t *ids, int64_t n_bins, int64_t *counts,
                             int32_t n_threads) {
    return guarded("igr_count_ids", [&]() -> int {
        const char *fn = "igr_count_ids";
        if (n < 0 || n_bins < 0 || (n > 0 && !ids) || (n_bins > 0 && !counts)) return arg_error(fn, "bad args");
        const int nt = resolve_threads(n_threads);
        std::memset(counts, 0, sizeof(int64_t) * (size_t)n_bins);
        std::atomic<int64_t> bad{-1};
        parallel_for(n, nt, [&](int64_t b, int64_t e) {
            for (int64_t i = b; i < e; ++i) {
                const int64_t k = ids[i];
                if (k < 0 || k >= n_bins) {
                    bad.store(i);
                    return;
                }
                __atomic_fetch_add(&counts[k], 1, __ATOMIC_RELAXED);
            }
        });
        if (bad.load() >= 0) return arg_error(fn, "id out of range at position " + std::to_string(bad.load()));
        return IGR_OK;
    });
}

extern "C" int igr_select_id_range(int64_t n, const int64_t *key, const int64_t *other, int64_t lo, int64_t hi,
                                   int64_t *out_key, int64_t *out_other, int64_t *n_out, int32_t n_threads) {
    return guarded("igr_select_id_range", [&]() -> int {
        const char *fn = "igr_select_id_range";
        if (n < 0 || !n_out || (n > 0 && !key)) return arg_error(fn, "bad args");
        if ((out_key == nullptr) != (out_other == nullptr) || (out_other && !other))
            return arg_error(fn, "out_key / out_other (and other) go together");
        // slices of the stream, one per thread: count, offsets, then an in-order copy
        const int nt = std::max(1, resolve_threads(n_threads));
        const int64_t step = (n + nt - 1) / nt;
        std::vector<int64_t> cnt(nt + 1, 0);
        per_thread(nt, [&](int t) {
            int64_t c = 0;
            for (int64_t i = t * step, e = std::min(n, (t + 1) * step); i < e; ++i) c += key[i] >= lo && key[i] < hi;
            cnt[t + 1] = c;
        });
        for (int t = 0; t < nt; ++t) cnt[t + 1] += cnt[t];
        *n_out = cnt[nt];
        if (!out_key) return IGR_OK;
        per_thread(nt, [&](int t) {
            int64_t o = cnt[t];
            for (int64_t i = t * step, e = std::min(n, (t + 1) * step); i < e; ++i)
                if (key[i] >= lo && key[i] < hi) {
                    out_key[o] = key[i] - lo;
                    out_other[o] = other[i];
                    ++o;
                }
        });
        return IGR_OK;
    });
}

extern "C" int igr_csr_transpose(int64_t n_rows, int64_t n_cols, const int64_t *row_ptr,
                                 const int32_t *col_idx, int64_t *t_row_ptr, int32_t *t_col_idx,
                                 int64_t *t_pos, int32_t n_threads) {
    return guarded("igr_csr_transpose", [&]() -> int {
        const char *fn = "igr_csr_transpose";
        if (n_rows < 0 || n_cols < 0) return arg_error(fn, "negative size");
        if (n_rows > INT32_MAX) return arg_error(fn, "n_rows exceeds int32 index");
        const int64_t nnz = row_ptr[n_rows];
        const int nt = resolve_threads(n_threads);
        std::vector<int64_t> cnt(n_cols, 0);
        parallel_for(nnz, nt, [&](int64_t b, int64_t e) {
            for (int64_t p = b; p < e; ++p) __atomic_fetch_add(&cnt[col_idx[p]], 1, __ATOMIC_RELAXED);
        });
        prefix(cnt.data(), n_cols, t_row_ptr);
        std::vector<int64_t> cur(t_row_ptr, t_row_ptr + n_cols);
        parallel_for(nnz, nt, [&](int64_t b, int64_t e) {
            for (int64_t p = b; p < e; ++p)
                t_pos[__atomic_fetch_add(&cur[col_idx[p]], 1, __ATOMIC_RELAXED)] = p;
        });
        // CSR positions increase with the row, so sorting positions sorts by source row
        parallel_for(n_cols, nt, [&](int64_t b, int64_t e) {
            for (int64_t c = b; c < e; ++c) std::sort(t_pos + t_row_ptr[c], t_pos + t_row_ptr[c + 1]);
        });
        // position -> row: each row's positions are contiguous
        std::vector<int32_t> prow(nnz);
        parallel_for(n_rows, nt, [&](int64_t b, int64_t e) {
            for (int64_t r = b; r < e; ++r)
                for (int64_t p = row_ptr[r]; p < row_ptr[r + 1]; ++p) prow[p] = (int32_t)r;
        });
        parallel_for(nnz, nt, [&](int64_t b, int64_t e) {
            for (int64_t q = b; q < e; ++q) t_col_idx[q] = prow[t_pos[q]];
        });
        return IGR_OK;
    });
}

extern "C" int igr_csr_row_sums(int64_t n_rows, const int64_t *row_ptr, const float *val, float *out) {
    return guarded("igr_csr_row_sums", [&]() -> int {
        if (n_rows < 0 || !row_ptr || !out) return arg_error("igr_csr_row_sums", "bad args");
        parallel_for(n_rows, resolve_threads(0), [&](int64_t b, int64_t e) {
            for (int64_t r = b; r < e; ++r) {
                float s = 0.f;  // fp32, CSR order (scipy's csr sum for float32)
                for (int64_t p = row_ptr[r]; p < row_ptr[r + 1]; ++p) s += val ? val[p] : 1.f;
                out[r] = s;
            }
        });
        return IGR_OK;
    });
}

extern "C" int igr_sym_norm_values(int64_t n_rows, const int64_t *row_ptr, const int32_t *col_idx,
                                   const float *val, const float *dinv_row, const float *dinv_col,
                                   float *out) {
    return guarded("igr_sym_norm_values", [&]() -> int {
        if (n_rows < 0 || !row_ptr || !dinv_row || !dinv_col || !out)
            return arg_error("igr_sym_norm_values", "bad args");
        parallel_for(n_rows, resolve_threads(0), [&](int64_t b, int64_t e) {
            for (int64_t r = b; r < e; ++r)
                for (int64_t p = row_ptr[r]; p < row_ptr[r + 1]; ++p) {
                    // sp.diags(dinv).dot(A).dot(sp.diags(dinv)) (model.py:95): (dinv_r * a) * dinv_c
                    const float t = dinv_row[r] * (val ? val[p] : 1.f);
                    out[p] = t * dinv_col[col_idx[p]];
                }
        });
        return IGR_OK;
    });
}

// ---------------------------------------------------------------- row schedule
namespace igr {

struct PlanCounts {
    int64_t n_order = 0, n_split = 0, n_chunks = 0;
};

static PlanCounts plan_counts(int64_t n_rows, const int64_t *row_ptr, int64_t thr, int64_t chunk) {
    PlanCounts c;
    for (int64_t r = 0; r < n_rows; ++r) {
        const int64_t deg = row_ptr[r + 1] - row_ptr[r];
        if (deg > thr) {
            ++c.n_split;
            c.n_chunks += (deg + chunk - 1) / chunk;
        } else {
            ++c.n_order;
        }
    }
    return c;
}

}  // namespace igr

extern "C" int igr_plan_size(int64_t n_rows, const int64_t *row_ptr, int64_t split_threshold,
                             int64_t chunk_edges, int64_t *n_order, int64_t *n_split,
                             int64_t *n_chunks) {
    return guarded("igr_plan_size", [&]() -> int {
        if (n_rows < 0 || !row_ptr || split_threshold < 1 || chunk_edges < 64 || chunk_edges % 64)
            return arg_error("igr_plan_size", "need split_threshold >= 1 and chunk_edges a multiple of 64");
        if (n_rows > INT32_MAX) return arg_error("igr_plan_size", "n_rows exceeds int32 row index");
        PlanCounts c = plan_counts(n_rows, row_ptr, split_threshold, chunk_edges);
        *n_order = c.n_order;
        *n_split = c.n_split;
        *n_chunks = c.n_chunks;
        return IGR_OK;
    });
}

extern "C" int igr_plan_fill(int64_t n_rows, const int64_t *row_ptr, int64_t split_threshold,
                             int64_t chunk_edges, int64_t window, int32_t *order, int32_t *split_row,
                             int64_t *split_ptr, int32_t *chunk_row, int64_t *chunk_beg) {
    return guarded("igr_plan_fill", [&]() -> int {
        if (n_rows < 0 || !row_ptr || split_threshold < 1 || chunk_edges < 64 || chunk_edges % 64 || window < 0)
            return arg_error("igr_plan_fill", "bad args");
        const int64_t thr = split_threshold;
        const int64_t win = window > 0 ? window : std::max<int64_t>(n_rows, 1);
        // Short rows: counting sort by degree, descending, inside windows of `win`
        // consecutive rows (ties by row id).  Windows keep the row_ptr reads and
        // output writes of one stretch of the launch inside an L2-sized range;
        // window = 0 sorts globally (heaviest first over the whole graph).
        std::vector<int64_t> bucket(thr + 2);
        std::vector<int32_t> longs;
        int64_t o = 0;
        for (int64_t w0 = 0; w0 < n_rows; w0 += win) {
            const int64_t w1 = std::min(n_rows, w0 + win);
            std::fill(bucket.begin(), bucket.end(), 0);
            for (int64_t r = w0; r < w1; ++r) {
                const int64_t deg = row_ptr[r + 1] - row_ptr[r];
                if (deg > thr) longs.push_back((int32_t)r);
                else bucket[thr - deg + 1]++;
            }
            bucket[0] = o;
            for (int64_t i = 0; i <= thr; ++i) bucket[i + 1] += bucket[i];
            for (int64_t r = w0; r < w1; ++r) {
                const int64_t deg = row_ptr[r + 1] - row_ptr[r];
                if (deg <= thr) order[bucket[thr - deg]++] = (int32_t)r;
            }
            o = bucket[thr];
        }
        // long rows: globally heaviest first, dispatched before every short row
        std::stable_sort(longs.begin(), longs.end(), [&](int32_t a, int32_t b) {
            return row_ptr[a + 1] - row_ptr[a] > row_ptr[b + 1] - row_ptr[b];
        });
        int64_t c = 0;
        if (split_ptr) split_ptr[0] = 0;
        for (size_t s = 0; s < longs.size(); ++s) {
            const int32_t r = longs[s];
            split_row[s] = r;
            for (int64_t p = row_ptr[r]; p < row_ptr[r + 1]; p += chunk_edges) {
                chunk_row[c] = r;
                chunk_beg[c] = p;
                ++c;
            }
            split_ptr[s + 1] = c;
        }
        return IGR_OK;
    });
}
