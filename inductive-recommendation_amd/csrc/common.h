// common.h - shared helpers for the igr HIP library (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <exception>
#include <string>

#include "igr.h"

namespace igr {

void set_error(const std::string &msg);

// Run `body`, converting exceptions to an error code (no exception crosses the C ABI).
template <class F>
int guarded(const char *fn, F &&body) {
    try {
        return body();
    } catch (const std::exception &e) {
        set_error(std::string(fn) + ": " + e.what());
        return IGR_ERR_INTERNAL;
    } catch (...) {
        set_error(std::string(fn) + ": unknown exception");
        return IGR_ERR_INTERNAL;
    }
}

inline int arg_error(const char *fn, const std::string &what) {
    set_error(std::string(fn) + ": " + what);
    return IGR_ERR_ARG;
}

inline int launch_status(const char *fn) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error(std::string(fn) + ": " + hipGetErrorString(e));
        return IGR_ERR_HIP;
    }
    return IGR_OK;
}

inline bool aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

constexpr int kWave = 64;  // CDNA wavefront

// The row schedule of a graph as the per-edge kernels use it (scores, dropout draws: an
// edge's result depends on no other edge, so the chunks of a split row need no combining):
// a wave takes one chunk of a split row or one whole unsplit row, heaviest first.
struct RowPlan {
    int64_t n_chunks;
    const int32_t *chunk_row;
    const int64_t *chunk_beg;
    int64_t chunk_edges;
    int64_t n_order;
    const int32_t *order;
};

inline RowPlan row_plan_of(const igr_csr *g) {
    return RowPlan{g->n_chunks, g->chunk_row, g->chunk_beg, g->chunk_edges, g->n_order, g->order};
}

// A graph carries a usable schedule when its unsplit-row list and its chunk list are both
// there (igr_plan_fill) and cover something.
// It must also cover every row exactly once (unsplit rows + split rows = rows) and name
// its split rows: a kernel that walks a partial plan would leave rows unwritten.
inline bool has_row_plan(const igr_csr *g) {
    if (g->n_order + g->n_chunks <= 0) return false;
    if (g->n_order + g->n_split != g->n_rows) return false;
    if (g->n_order > 0 && !g->order) return false;
    if (g->n_chunks > 0 && (!g->chunk_row || !g->chunk_beg || g->chunk_edges <= 0)) return false;
    if ((g->n_split > 0) != (g->n_chunks > 0)) return false;
    if (g->n_split > 0 && (!g->split_row || !g->split_ptr)) return false;
    return true;
}

// The plan is used where it pays: when rows were split (skewed degrees: a hub row would
// otherwise be one wave's serial loop) or when the graph is small enough for a launch to
// last as long as its heaviest row (heaviest first).  On a large graph of alike rows the
// natural row order streams the per-row operands better (SDDMM at nnz 411 M, h = 4,
// d = 64: 19.8 ms against 20.4).
inline bool use_row_plan(const igr_csr *g) {
    return has_row_plan(g) && (g->n_chunks > 0 || g->n_rows <= (1 << 18));
}

}  // namespace igr

// ---------------------------------------------------------------- device helpers
#ifdef __HIPCC__
namespace igr {

__device__ __forceinline__ float4 f4_fma(float w, float4 x, float4 a) {
    a.x = fmaf(w, x.x, a.x);
    a.y = fmaf(w, x.y, a.y);
    a.z = fmaf(w, x.z, a.z);
    a.w = fmaf(w, x.w, a.w);
    return a;
}

__device__ __forceinline__ float4 f4_add(float4 a, float4 b) {
    return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

__device__ __forceinline__ float4 f4_scale(float s, float4 a) {
    return make_float4(s * a.x, s * a.y, s * a.z, s * a.w);
}

__device__ __forceinline__ float4 f4_div(float4 a, float s) {
    return make_float4(a.x / s, a.y / s, a.z / s, a.w / s);
}

// Streamed-once loads (CSR structure, edge values).  Measured on MI355X
// (scripts/tune_spmm.py, 10M x 1M d=64): plain loads are 1-3 % faster than
// non-temporal ones here, so IGR_NT_STREAM_LOADS is off by default.
#ifdef IGR_NT_STREAM_LOADS
template <class T>
__device__ __forceinline__ T ld_stream(const T *p) {
    return __builtin_nontemporal_load(p);
}
#else
template <class T>
__device__ __forceinline__ T ld_stream(const T *p) {
    return *p;
}
#endif

// Counter-based random numbers: splitmix64 finaliser of (seed, offset, index).
// A draw is a pure function of its counters, so a kernel needs no RNG state
// and a backward pass can regenerate exactly the forward's draws.
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ uint64_t draw64(uint64_t seed, uint64_t offset, uint64_t i, uint32_t round) {
    return mix64(mix64(seed ^ mix64(offset)) + (i << 8) + round);
}

// U[0, 1) with 24 random bits (the resolution of torch.rand for float32).
__device__ __forceinline__ float uniform24(uint64_t seed, uint64_t offset, uint64_t i) {
    return (float)(draw64(seed, offset, i, 0xD7) >> 40) * (1.0f / 16777216.0f);
}

// Lane shuffle within the wave (ds_bpermute).
__device__ __forceinline__ int shfl_i(int v, int src) { return __shfl(v, src, 64); }
__device__ __forceinline__ int64_t shfl_i64(int64_t v, int src) {
    return ((int64_t)__shfl((int)(v >> 32), src, 64) << 32) | (uint32_t)__shfl((int)v, src, 64);
}
__device__ __forceinline__ float shfl_f(float v, int src) { return __shfl(v, src, 64); }
__device__ __forceinline__ float shfl_xor_f(float v, int m) { return __shfl_xor(v, m, 64); }

}  // namespace igr
#endif
