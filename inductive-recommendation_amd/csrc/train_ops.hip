// train_ops.hip - the training step around the propagation (gfx950):
//
//   igr_bpr_sample          device-side BPR negative sampler      dataset.py:119-131
//                           (replaces the CPU sampler in 6 DataLoader workers + H2D,
//                            trainer.py:522-535)
//   igr_adam_f32            fused Adam update, torch.optim.Adam    trainer.py:44-46, 555
//                           semantics in one pass
#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "common.h"

namespace igr {

__device__ __forceinline__ uint64_t draw(uint64_t seed, uint64_t offset, uint64_t i, uint32_t round) {
    return draw64(seed, offset, i, round);
}

// uniform integer in [0, n) from 64 random bits (Lemire's multiply-shift; bias < n / 2^64)
__device__ __forceinline__ int64_t bounded(uint64_t r, int64_t n) {
    return (int64_t)(((unsigned __int128)r * (uint64_t)n) >> 64);
}

// true if `item` is in the sorted list items[b, e)
__device__ __forceinline__ bool member(const int32_t *__restrict__ items, int64_t b, int64_t e, int32_t item) {
    while (b < e) {
        const int64_t m = (b + e) >> 1;
        const int32_t v = items[m];
        if (v == item) return true;
        if (v < item) b = m + 1;
        else e = m;
    }
    return false;
}

__global__ void bpr_sample_kernel(int64_t batch, int64_t n_active, const int32_t *__restrict__ active,
                                  const int64_t *__restrict__ row_ptr, const int32_t *__restrict__ items,
                                  int64_t n_items, uint64_t seed, uint64_t offset0,
                                  const int64_t *__restrict__ offset_dev, int32_t max_rounds,
                                  int64_t *__restrict__ users, int64_t *__restrict__ pos,
                                  int64_t *__restrict__ neg) {
    const uint64_t offset = offset0 + (offset_dev ? (uint64_t)*offset_dev : 0);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < batch;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t u = active[bounded(draw(seed, offset, i, 0), n_active)];
        const int64_t b = row_ptr[u], e = row_ptr[u + 1];
        const int32_t p = items[b + bounded(draw(seed, offset, i, 1), e - b)];
        int32_t n = (int32_t)bounded(draw(seed, offset, i, 2), n_items);
        // rejection as dataset.py:126-128; bounded so a user who interacted with
        // every item cannot spin forever (the reference would): such a user keeps
        // the last draw, every other user always ends with a true negative
        int32_t k = 3;
        for (; k < max_rounds + 3 && member(items, b, e, n); ++k)
            n = (int32_t)bounded(draw(seed, offset, i, (uint32_t)k), n_items);
        if (k == max_rounds + 3 && member(items, b, e, n) && (e - b) < n_items) {
            // every redraw hit the user's own list (a heavy user of a small item set):
            // take the j-th item of the complement directly, j uniform.  The sorted list
            // has items[b + c] - c non-decreasing, so the number c of list items before
            // the j-th gap is found by bisection and the answer is j + c.
            const int64_t j = bounded(draw(seed, offset, i, (uint32_t)k), n_items - (e - b));
            int64_t lo = 0, hi = e - b;
            while (lo < hi) {
                const int64_t m = (lo + hi) >> 1;
                if ((int64_t)items[b + m] - m <= j) lo = m + 1;
                else hi = m;
            }
            n = (int32_t)(j + lo);
        }
        users[i] = u;
        pos[i] = p;
        neg[i] = n;
    }
}

// torch.optim.Adam single-tensor semantics (torch/optim/adam.py, non-amsgrad,
// non-capturable):  m.lerp_(g, 1-b1); v = v*b2 + (1-b2) g^2;
// p -= (lr / bc1) * m / (sqrt(v) / sqrt(bc2) + eps); weight_decay adds wd*p to g.
// omb1 = 1 - beta1 and omb2 = 1 - beta2 are formed in double on the host, as
// torch forms them from Python floats.
// step_dev (hipGraph-capturable form): the step is step0 + *step_dev, read on the
// device, and the bias corrections are formed from it in double here.
typedef float v4f __attribute__((ext_vector_type(4)));
__device__ __forceinline__ v4f to_v4(float4 a) { return v4f{a.x, a.y, a.z, a.w}; }
__device__ __forceinline__ float4 from_v4(v4f a) { return make_float4(a.x, a.y, a.z, a.w); }

template <int U, bool NT>
__global__ void adam_kernel(int64_t n, float *__restrict__ p, const float *__restrict__ g,
                            float *__restrict__ m, float *__restrict__ v, float omb1, float b2, float omb2,
                            float eps, float wd, float step_size, float bc2_sqrt,
                            const int64_t *__restrict__ step_dev, int64_t step0, double lr, double beta1,
                            double beta2) {
    if (step_dev) {
        const double t = (double)(step0 + *step_dev);
        step_size = (float)(lr / (1.0 - pow(beta1, t)));
        bc2_sqrt = (float)sqrt(1.0 - pow(beta2, t));
    }
    const int64_t n4 = n >> 2;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    // U float4 of each array per thread per trip, all loads issued before the math
    for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < n4; i0 += stride * U) {
        float4 pp[U], gg[U], mm[U], vv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = i0 + u * stride;
            if (i < n4) {
                pp[u] = reinterpret_cast<float4 *>(p)[i];
                gg[u] = NT ? from_v4(__builtin_nontemporal_load(reinterpret_cast<const v4f *>(g) + i))
                           : reinterpret_cast<const float4 *>(g)[i];
                mm[u] = reinterpret_cast<float4 *>(m)[i];
                vv[u] = reinterpret_cast<float4 *>(v)[i];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = i0 + u * stride;
            if (i >= n4) break;
            float *pa = &pp[u].x, *ga = &gg[u].x, *ma = &mm[u].x, *va = &vv[u].x;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float gk = wd != 0.f ? ga[k] + wd * pa[k] : ga[k];
                ma[k] = ma[k] + omb1 * (gk - ma[k]);
                va[k] = va[k] * b2 + omb2 * gk * gk;
                const float den = sqrtf(va[k]) / bc2_sqrt + eps;
                pa[k] = pa[k] - step_size * (ma[k] / den);
            }
            if (NT) {
                __builtin_nontemporal_store(to_v4(pp[u]), reinterpret_cast<v4f *>(p) + i);
                __builtin_nontemporal_store(to_v4(mm[u]), reinterpret_cast<v4f *>(m) + i);
                __builtin_nontemporal_store(to_v4(vv[u]), reinterpret_cast<v4f *>(v) + i);
            } else {
                reinterpret_cast<float4 *>(p)[i] = pp[u];
                reinterpret_cast<float4 *>(m)[i] = mm[u];
                reinterpret_cast<float4 *>(v)[i] = vv[u];
            }
        }
    }
    for (int64_t i = 4 * n4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const float gk = wd != 0.f ? g[i] + wd * p[i] : g[i];
        m[i] = m[i] + omb1 * (gk - m[i]);
        v[i] = v[i] * b2 + omb2 * gk * gk;
        p[i] = p[i] - step_size * (m[i] / (sqrtf(v[i]) / bc2_sqrt + eps));
    }
}

// The same update for up to IGR_ADAM_MAX_SLOTS small tensors in ONE launch (a model's
// projection weights, biases and feature weights: a launch each costs more than their
// arithmetic).  Workgroup b serves 1024 elements of the slot whose block range holds b;
// the arithmetic is adam_kernel's, expression for expression, so the bits are the same.
struct AdamMulti {
    float *p[IGR_ADAM_MAX_SLOTS];
    const float *g[IGR_ADAM_MAX_SLOTS];
    float *m[IGR_ADAM_MAX_SLOTS];
    float *v[IGR_ADAM_MAX_SLOTS];
    int64_t n[IGR_ADAM_MAX_SLOTS];
    int64_t step0[IGR_ADAM_MAX_SLOTS];
    float step_size[IGR_ADAM_MAX_SLOTS];
    float bc2_sqrt[IGR_ADAM_MAX_SLOTS];
    int32_t blk0[IGR_ADAM_MAX_SLOTS + 1];
};

__global__ __launch_bounds__(256) void adam_multi_kernel(AdamMulti a, int n_slots, float omb1, float b2, float omb2,
                                                         float eps, float wd, const int64_t *__restrict__ step_dev,
                                                         double lr, double beta1, double beta2) {
    int k = 0;
    while (k + 1 < n_slots && (int)blockIdx.x >= a.blk0[k + 1]) ++k;
    float step_size = a.step_size[k], bc2_sqrt = a.bc2_sqrt[k];
    if (step_dev) {
        const double t = (double)(a.step0[k] + *step_dev);
        step_size = (float)(lr / (1.0 - pow(beta1, t)));
        bc2_sqrt = (float)sqrt(1.0 - pow(beta2, t));
    }
    float *__restrict__ p = a.p[k];
    const float *__restrict__ g = a.g[k];
    float *__restrict__ m = a.m[k];
    float *__restrict__ v = a.v[k];
    const int64_t n = a.n[k], n4 = n >> 2;
    const int64_t i = (int64_t)((int)blockIdx.x - a.blk0[k]) * 256 + threadIdx.x;  // float4 index
    if (i < n4) {
        float4 pp = reinterpret_cast<float4 *>(p)[i], gg = reinterpret_cast<const float4 *>(g)[i];
        float4 mm = reinterpret_cast<float4 *>(m)[i], vv = reinterpret_cast<float4 *>(v)[i];
        float *pa = &pp.x, *ga = &gg.x, *ma = &mm.x, *va = &vv.x;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float gk = wd != 0.f ? ga[q] + wd * pa[q] : ga[q];
            ma[q] = ma[q] + omb1 * (gk - ma[q]);
            va[q] = va[q] * b2 + omb2 * gk * gk;
            const float den = sqrtf(va[q]) / bc2_sqrt + eps;
            pa[q] = pa[q] - step_size * (ma[q] / den);
        }
        reinterpret_cast<float4 *>(p)[i] = pp;
        reinterpret_cast<float4 *>(m)[i] = mm;
        reinterpret_cast<float4 *>(v)[i] = vv;
    }
    // the last n % 4 elements: the slot's first workgroup
    const int64_t j = 4 * n4 + threadIdx.x;
    if ((int)blockIdx.x == a.blk0[k] && j < n) {
        const float gk = wd != 0.f ? g[j] + wd * p[j] : g[j];
        m[j] = m[j] + omb1 * (gk - m[j]);
        v[j] = v[j] * b2 + omb2 * gk * gk;
        p[j] = p[j] - step_size * (m[j] / (sqrtf(v[j]) / bc2_sqrt + eps));
    }
}

static unsigned grid_for(int64_t n, int block) {
    int64_t g = (n + block - 1) / block;
    if (g > 16384) g = 16384;
    return (unsigned)(g < 1 ? 1 : g);
}

}  // namespace igr

using namespace igr;

extern "C" int igr_bpr_sample(int64_t batch, int64_t n_active, const int32_t *active, const int64_t *row_ptr,
                              const int32_t *items, int64_t n_items, uint64_t seed, uint64_t offset,
                              const int64_t *offset_dev, int32_t max_rounds, int64_t *users, int64_t *pos,
                              int64_t *neg, void *stream) {
    return guarded("igr_bpr_sample", [&]() -> int {
        if (n_active <= 0 || n_items <= 0) return arg_error("igr_bpr_sample", "no active users / items");
        if (max_rounds < 0) return arg_error("igr_bpr_sample", "max_rounds < 0");
        if (batch <= 0) return IGR_OK;
        hipStream_t st = reinterpret_cast<hipStream_t>(stream);
        hipLaunchKernelGGL(bpr_sample_kernel, dim3(grid_for(batch, 256)), dim3(256), 0, st, batch, n_active,
                           active, row_ptr, items, n_items, seed, offset, offset_dev, max_rounds, users, pos,
                           neg);
        return launch_status("igr_bpr_sample");
    });
}

extern "C" int igr_adam_f32(int64_t n, float *param, const float *grad, float *exp_avg, float *exp_avg_sq,
                            double lr, double beta1, double beta2, double eps, double weight_decay, int64_t step,
                            const int64_t *step_dev, void *stream) {
    return guarded("igr_adam_f32", [&]() -> int {
        if (step < (step_dev ? 0 : 1)) return arg_error("igr_adam_f32", "step must be >= 1");
        if (n <= 0) return IGR_OK;
        if (!aligned16(param) || !aligned16(grad) || !aligned16(exp_avg) || !aligned16(exp_avg_sq))
            return arg_error("igr_adam_f32", "buffers must be 16-byte aligned");
        // bias corrections in double on the host, as torch computes them from Python floats
        const double bc1 = step_dev ? 1.0 : 1.0 - std::pow(beta1, (double)step);
        const double bc2 = step_dev ? 1.0 : 1.0 - std::pow(beta2, (double)step);
        const float step_size = (float)(lr / bc1);
        const float bc2_sqrt = (float)std::sqrt(bc2);
        hipStream_t st = reinterpret_cast<hipStream_t>(stream);
        const float omb1 = (float)(1.0 - beta1), omb2 = (float)(1.0 - beta2);
        // one float4 of each array per thread, no grid cap, non-temporal traffic: the best of
        // the sweep over float4s per thread x grid cap x temporal hint on the 70 M-parameter
        // table (5.15 -> 5.7 TB/s, profiles/r01m_adam_sweep.json); the wider variants spilled
        const int64_t grid = std::max<int64_t>(std::min<int64_t>(((n + 3) / 4 + 255) / 256, int64_t(1) << 30), 1);
        hipLaunchKernelGGL((adam_kernel<1, true>), dim3((unsigned)grid), dim3(256), 0, st, n, param, grad, exp_avg,
                           exp_avg_sq, omb1, (float)beta2, omb2, (float)eps, (float)weight_decay, step_size, bc2_sqrt,
                           step_dev, step, lr, beta1, beta2);
        return launch_status("igr_adam_f32");
    });
}

extern "C" int igr_adam_multi_f32(int32_t n_slots, const igr_adam_slot *slots, double lr, double beta1, double beta2,
                                  double eps, double weight_decay, const int64_t *step_dev, void *stream) {
    return guarded("igr_adam_multi_f32", [&]() -> int {
        const char *fn = "igr_adam_multi_f32";
        if (n_slots < 0 || n_slots > IGR_ADAM_MAX_SLOTS) return arg_error(fn, "0 <= n_slots <= IGR_ADAM_MAX_SLOTS");
        if (n_slots == 0) return IGR_OK;
        if (!slots) return arg_error(fn, "NULL slots");
        AdamMulti a;
        int64_t blocks = 0;
        for (int k = 0; k < n_slots; ++k) {
            const igr_adam_slot &s = slots[k];
            if (s.n <= 0 || s.n > (int64_t(1) << 30)) return arg_error(fn, "slot size must be in (0, 2^30]");
            if (s.step < (step_dev ? 0 : 1)) return arg_error(fn, "step must be >= 1");
            if (!s.param || !s.grad || !s.exp_avg || !s.exp_avg_sq) return arg_error(fn, "NULL pointer in a slot");
            if (!aligned16(s.param) || !aligned16(s.grad) || !aligned16(s.exp_avg) || !aligned16(s.exp_avg_sq))
                return arg_error(fn, "buffers must be 16-byte aligned");
            const double bc1 = step_dev ? 1.0 : 1.0 - std::pow(beta1, (double)s.step);
            const double bc2 = step_dev ? 1.0 : 1.0 - std::pow(beta2, (double)s.step);
            a.p[k] = s.param, a.g[k] = s.grad, a.m[k] = s.exp_avg, a.v[k] = s.exp_avg_sq;
            a.n[k] = s.n, a.step0[k] = s.step;
            a.step_size[k] = (float)(lr / bc1), a.bc2_sqrt[k] = (float)std::sqrt(bc2);
            a.blk0[k] = (int32_t)blocks;
            blocks += std::max<int64_t>(1, ((s.n >> 2) + 255) / 256);
            if (blocks > 2147483647) return arg_error(fn, "too many elements for one launch");
        }
        a.blk0[n_slots] = (int32_t)blocks;
        hipLaunchKernelGGL(adam_multi_kernel, dim3((unsigned)blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                           a, (int)n_slots, (float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2), (float)eps,
                           (float)weight_decay, step_dev, lr, beta1, beta2);
        return launch_status(fn);
    });
}

namespace igr {
__global__ void counter_add_kernel(int64_t *ctr, int64_t v) {
    if (threadIdx.x == 0) *ctr += v;
}
}  // namespace igr

extern "C" int igr_counter_add(int64_t *counter, int64_t value, void *stream) {
    return guarded("igr_counter_add", [&]() -> int {
        if (!counter) return arg_error("igr_counter_add", "counter is NULL");
        hipLaunchKernelGGL(counter_add_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), counter,
                           value);
        return launch_status("igr_counter_add");
    });
}

// ---- NGCF layer tail (model.py:4040-4042): r = dropout(leaky_relu(a + b)), nrm = r / max(|r|_2, eps)
// One wave per node row, lane l holds columns l, l + 64, ... (V of them): one coalesced read of
// a and b, one write of r and nrm; the row norm is a wave reduction.  keep (0/1 per element,
// NULL in eval mode) times keep_scale = 1 / (1 - p) is the dropout mask.
namespace igr {

constexpr float kNormEps = 1e-12f;  // F.normalize's eps

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += shfl_xor_f(v, m);
    return v;
}

template <int V>
__global__ __launch_bounds__(256) void layer_tail_kernel(int64_t n, int d, const float *__restrict__ a, int64_t lda,
                                                         const float *__restrict__ b, int64_t ldb,
                                                         const float *__restrict__ keep, float keep_scale, float slope,
                                                         float *__restrict__ r, float *__restrict__ nrm, int64_t ldn,
                                                         float *__restrict__ row_norm) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= n) return;  // whole waves leave; no barrier below
    float y[V];
    float ss = 0.f;
#pragma unroll
    for (int v = 0; v < V; ++v) {
        const int c = lane + 64 * v;
        y[v] = 0.f;
        if (c < d) {
            const float z = a[row * lda + c] + b[row * ldb + c];
            float t = z > 0.f ? z : z * slope;
            if (keep) t = t * keep[row * d + c] * keep_scale;
            y[v] = t;
            ss += t * t;
        }
    }
    const float nr = fmaxf(sqrtf(wave_sum(ss)), kNormEps);
#pragma unroll
    for (int v = 0; v < V; ++v) {
        const int c = lane + 64 * v;
        if (c < d) {
            r[row * d + c] = y[v];
            nrm[row * ldn + c] = y[v] / nr;
        }
    }
    if (lane == 0) row_norm[row] = nr;
}

// gradient of the tail: gn = d loss / d nrm, gr = d loss / d r (either may be NULL), both added;
// dz = d loss / d (a + b).  The normalisation's clamp passes no gradient through the norm.
template <int V>
__global__ __launch_bounds__(256) void layer_tail_bwd_kernel(int64_t n, int d, const float *__restrict__ gn, int64_t ldgn,
                                                             const float *__restrict__ gr, int64_t ldgr,
                                                             const float *__restrict__ r,
                                                             const float *__restrict__ row_norm,
                                                             const float *__restrict__ keep, float keep_scale,
                                                             float slope, float *__restrict__ dz) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= n) return;
    const float nr = row_norm[row];
    float rv[V], g[V];
    float dot = 0.f;
#pragma unroll
    for (int v = 0; v < V; ++v) {
        const int c = lane + 64 * v;
        rv[v] = g[v] = 0.f;
        if (c < d) {
            rv[v] = r[row * d + c];
            if (gn) {
                g[v] = gn[row * ldgn + c];
                dot += g[v] * rv[v];
            }
        }
    }
    // nrm = r / nr: d/dr = (gn - nrm <gn, nrm>) / nr above the clamp, gn / nr on it
    const float proj = nr > kNormEps ? wave_sum(dot) / (nr * nr) : 0.f;
#pragma unroll
    for (int v = 0; v < V; ++v) {
        const int c = lane + 64 * v;
        if (c < d) {
            float t = gn ? (g[v] - rv[v] * proj) / nr : 0.f;
            if (gr) t += gr[row * ldgr + c];
            if (keep) t = t * keep[row * d + c] * keep_scale;
            dz[row * d + c] = rv[v] > 0.f ? t : t * slope;
        }
    }
}

// The same two kernels for d = 4 LPR (d = 32, 64, 128, 256) with 16-byte aligned rows: LPR
// lanes hold one row as float4s, 64 / LPR rows per wave, so every load and store instruction
// moves whole 16-byte pieces (the one-float-per-lane form reads a 256-byte row with 64 lanes).
typedef float tail_f4 __attribute__((ext_vector_type(4)));

template <int LPR>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
    for (int m = LPR / 2; m >= 1; m >>= 1) v += shfl_xor_f(v, m);
    return v;
}

template <int LPR>
__global__ __launch_bounds__(256) void layer_tail_vec_kernel(int64_t n, const float *__restrict__ a, int64_t lda,
                                                             const float *__restrict__ b, int64_t ldb,
                                                             const float *__restrict__ keep, float keep_scale,
                                                             float slope, float *__restrict__ r,
                                                             float *__restrict__ nrm, int64_t ldn,
                                                             float *__restrict__ row_norm) {
    constexpr int RPW = 64 / LPR, D = 4 * LPR;
    const int lane = threadIdx.x & 63, sub = lane % LPR;
    const int64_t row = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW + lane / LPR;
    const bool live = row < n;
    const int64_t rr = live ? row : n - 1;  // every lane stays for the shuffles; dead rows are not stored
    const tail_f4 av = *reinterpret_cast<const tail_f4 *>(a + rr * lda + 4 * sub);
    const tail_f4 bv = *reinterpret_cast<const tail_f4 *>(b + rr * ldb + 4 * sub);
    tail_f4 y;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const float z = av[q] + bv[q];
        y[q] = z > 0.f ? z : z * slope;
    }
    if (keep) {
        const tail_f4 kv = *reinterpret_cast<const tail_f4 *>(keep + rr * D + 4 * sub);
#pragma unroll
        for (int q = 0; q < 4; ++q) y[q] = y[q] * kv[q] * keep_scale;
    }
    const float ss = group_sum<LPR>(y[0] * y[0] + y[1] * y[1] + y[2] * y[2] + y[3] * y[3]);
    const float nr = fmaxf(sqrtf(ss), kNormEps);
    if (!live) return;
    *reinterpret_cast<tail_f4 *>(r + row * D + 4 * sub) = y;
    *reinterpret_cast<tail_f4 *>(nrm + row * ldn + 4 * sub) = tail_f4{y[0] / nr, y[1] / nr, y[2] / nr, y[3] / nr};
    if (sub == 0) row_norm[row] = nr;
}

template <int LPR>
__global__ __launch_bounds__(256) void layer_tail_bwd_vec_kernel(int64_t n, const float *__restrict__ gn, int64_t ldgn,
                                                                 const float *__restrict__ gr, int64_t ldgr,
                                                                 const float *__restrict__ r,
                                                                 const float *__restrict__ row_norm,
                                                                 const float *__restrict__ keep, float keep_scale,
                                                                 float slope, float *__restrict__ dz) {
    constexpr int RPW = 64 / LPR, D = 4 * LPR;
    const int lane = threadIdx.x & 63, sub = lane % LPR;
    const int64_t row = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW + lane / LPR;
    const bool live = row < n;
    const int64_t rr = live ? row : n - 1;
    const float nr = row_norm[rr];
    const tail_f4 rv = *reinterpret_cast<const tail_f4 *>(r + rr * D + 4 * sub);
    tail_f4 g = tail_f4{0.f, 0.f, 0.f, 0.f};
    float dot = 0.f;
    if (gn) {
        g = *reinterpret_cast<const tail_f4 *>(gn + rr * ldgn + 4 * sub);
        dot = g[0] * rv[0] + g[1] * rv[1] + g[2] * rv[2] + g[3] * rv[3];
    }
    dot = group_sum<LPR>(dot);
    const float proj = nr > kNormEps ? dot / (nr * nr) : 0.f;
    tail_f4 t = tail_f4{0.f, 0.f, 0.f, 0.f};
    if (gn) {
#pragma unroll
        for (int q = 0; q < 4; ++q) t[q] = (g[q] - rv[q] * proj) / nr;
    }
    if (gr) {
        const tail_f4 gv = *reinterpret_cast<const tail_f4 *>(gr + rr * ldgr + 4 * sub);
#pragma unroll
        for (int q = 0; q < 4; ++q) t[q] += gv[q];
    }
    if (keep) {
        const tail_f4 kv = *reinterpret_cast<const tail_f4 *>(keep + rr * D + 4 * sub);
#pragma unroll
        for (int q = 0; q < 4; ++q) t[q] = t[q] * kv[q] * keep_scale;
    }
    if (!live) return;
#pragma unroll
    for (int q = 0; q < 4; ++q) t[q] = rv[q] > 0.f ? t[q] : t[q] * slope;
    *reinterpret_cast<tail_f4 *>(dz + row * D + 4 * sub) = t;
}

}  // namespace igr

static bool tail_args_ok(const char *fn, int64_t n, int32_t d) {
    if (n < 0 || d <= 0 || d > 256) {
        arg_error(fn, "need n >= 0 and 0 < d <= 256");
        return false;
    }
    return true;
}

extern "C" int igr_layer_tail_f32(int64_t n, int32_t d, const float *a, int64_t lda, const float *b, int64_t ldb,
                                  const float *keep, float keep_scale, float slope, float *r, float *nrm, int64_t ldn,
                                  float *row_norm, void *stream) {
    return guarded("igr_layer_tail_f32", [&]() -> int {
        const char *fn = "igr_layer_tail_f32";
        if (!tail_args_ok(fn, n, d)) return IGR_ERR_ARG;
        if (n == 0) return IGR_OK;
        if (!a || !b || !r || !nrm || !row_norm) return arg_error(fn, "NULL pointer");
        if (lda < d || ldb < d || ldn < d) return arg_error(fn, "leading dimension too small");
        if ((n + 3) / 4 > 2147483647) return arg_error(fn, "too many rows");
        hipStream_t st = reinterpret_cast<hipStream_t>(stream);
        const bool vec = (d == 32 || d == 64 || d == 128 || d == 256) && lda % 4 == 0 && ldb % 4 == 0 &&
                         ldn % 4 == 0 && aligned16(a) && aligned16(b) && aligned16(r) && aligned16(nrm) &&
                         (!keep || aligned16(keep));
        if (vec) {
            const int64_t rows_per_block = 4 * (64 / (d / 4));
            const dim3 gv((unsigned)((n + rows_per_block - 1) / rows_per_block));
#define IGR_TAILV(L_)                                                                                              \
    hipLaunchKernelGGL((layer_tail_vec_kernel<L_>), gv, dim3(256), 0, st, n, a, lda, b, ldb, keep, keep_scale, slope, r, \
                       nrm, ldn, row_norm)
            if (d == 32) IGR_TAILV(8); else if (d == 64) IGR_TAILV(16); else if (d == 128) IGR_TAILV(32); else IGR_TAILV(64);
#undef IGR_TAILV
            return launch_status(fn);
        }
        const dim3 grid((unsigned)((n + 3) / 4));
#define IGR_TAIL(V_)                                                                                             \
    hipLaunchKernelGGL((layer_tail_kernel<V_>), grid, dim3(256), 0, st, n, (int)d, a, lda, b, ldb, keep, keep_scale, \
                       slope, r, nrm, ldn, row_norm)
        if (d <= 64) IGR_TAIL(1); else if (d <= 128) IGR_TAIL(2); else IGR_TAIL(4);
#undef IGR_TAIL
        return launch_status(fn);
    });
}

extern "C" int igr_layer_tail_bwd_f32(int64_t n, int32_t d, const float *gn, int64_t ldgn, const float *gr, int64_t ldgr,
                                      const float *r, const float *row_norm, const float *keep, float keep_scale,
                                      float slope, float *dz, void *stream) {
    return guarded("igr_layer_tail_bwd_f32", [&]() -> int {
        const char *fn = "igr_layer_tail_bwd_f32";
        if (!tail_args_ok(fn, n, d)) return IGR_ERR_ARG;
        if (n == 0) return IGR_OK;
        if (!r || !row_norm || !dz) return arg_error(fn, "NULL pointer");
        if ((gn && ldgn < d) || (gr && ldgr < d)) return arg_error(fn, "leading dimension too small");
        if ((n + 3) / 4 > 2147483647) return arg_error(fn, "too many rows");
        hipStream_t st = reinterpret_cast<hipStream_t>(stream);
        const bool vec = (d == 32 || d == 64 || d == 128 || d == 256) && aligned16(r) && aligned16(dz) &&
                         (!gn || (ldgn % 4 == 0 && aligned16(gn))) && (!gr || (ldgr % 4 == 0 && aligned16(gr))) &&
                         (!keep || aligned16(keep));
        if (vec) {
            const int64_t rows_per_block = 4 * (64 / (d / 4));
            const dim3 gv((unsigned)((n + rows_per_block - 1) / rows_per_block));
#define IGR_TAILBV(L_)                                                                                             \
    hipLaunchKernelGGL((layer_tail_bwd_vec_kernel<L_>), gv, dim3(256), 0, st, n, gn, ldgn, gr, ldgr, r, row_norm, keep, \
                       keep_scale, slope, dz)
            if (d == 32) IGR_TAILBV(8); else if (d == 64) IGR_TAILBV(16); else if (d == 128) IGR_TAILBV(32); else IGR_TAILBV(64);
#undef IGR_TAILBV
            return launch_status(fn);
        }
        const dim3 grid((unsigned)((n + 3) / 4));
#define IGR_TAILB(V_)                                                                                              \
    hipLaunchKernelGGL((layer_tail_bwd_kernel<V_>), grid, dim3(256), 0, st, n, (int)d, gn, ldgn, gr, ldgr, r, row_norm, \
                       keep, keep_scale, slope, dz)
        if (d <= 64) IGR_TAILB(1); else if (d <= 128) IGR_TAILB(2); else IGR_TAILB(4);
#undef IGR_TAILB
        return launch_status(fn);
    });
}
