// train_ops.hip - the training step around the propagation (gfx950):
//
//   igr_bpr_sample          device-side BPR negative sampler      dataset.py:119-131
//                           (replaces the CPU sampler in 6 DataLoader workers + H2D,
//                            trainer.py:522-535)
//   igr_adam_f32            fused Adam update, torch.optim.Adam    trainer.py:44-46, 555
//                           semantics in one pass
#include <cmath>

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
        // every item cannot spin forever (the reference would)
        for (int32_t k = 3; k < max_rounds + 3 && member(items, b, e, n); ++k)
            n = (int32_t)bounded(draw(seed, offset, i, (uint32_t)k), n_items);
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
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
        float4 pp = reinterpret_cast<float4 *>(p)[i];
        float4 gg = reinterpret_cast<const float4 *>(g)[i];
        float4 mm = reinterpret_cast<float4 *>(m)[i];
        float4 vv = reinterpret_cast<float4 *>(v)[i];
        float *pa = &pp.x, *ga = &gg.x, *ma = &mm.x, *va = &vv.x;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float gk = wd != 0.f ? ga[k] + wd * pa[k] : ga[k];
            ma[k] = ma[k] + omb1 * (gk - ma[k]);
            va[k] = va[k] * b2 + omb2 * gk * gk;
            const float den = sqrtf(va[k]) / bc2_sqrt + eps;
            pa[k] = pa[k] - step_size * (ma[k] / den);
        }
        reinterpret_cast<float4 *>(p)[i] = pp;
        reinterpret_cast<float4 *>(m)[i] = mm;
        reinterpret_cast<float4 *>(v)[i] = vv;
    }
    for (int64_t i = 4 * n4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const float gk = wd != 0.f ? g[i] + wd * p[i] : g[i];
        m[i] = m[i] + omb1 * (gk - m[i]);
        v[i] = v[i] * b2 + omb2 * gk * gk;
        p[i] = p[i] - step_size * (m[i] / (sqrtf(v[i]) / bc2_sqrt + eps));
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
        hipLaunchKernelGGL(adam_kernel, dim3(grid_for((n + 3) / 4, 256)), dim3(256), 0, st, n, param, grad,
                           exp_avg, exp_avg_sq, omb1, (float)beta2, omb2, (float)eps, (float)weight_decay, step_size, bc2_sqrt,
                           step_dev, step, lr, beta1, beta2);
        return launch_status("igr_adam_f32");
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
