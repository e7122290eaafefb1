// bpr.hip - BPR negative-sample embedding gathers and the fused BPR loss
// (gfx950).
//
//   igr_gather_rows_f32       rep[users], rep[n_users + pos/neg]   model.py:4048-4049
//   igr_scatter_add_rows_f32  their backward (index_put accumulate)
//   igr_bpr_fwd_bwd_f32       NGCF.bpr_forward + IGCNTrainer loss   model.py:4046-4052,
//                             (BPR term and the aux term with w)    trainer.py:536-549
#include "common.h"

namespace igr {

constexpr int kBprMaxD = 1024;  // LDS bound for the dw reduction

__global__ void gather_rows_kernel(int64_t n, int d, const int64_t *__restrict__ idx,
                                   int64_t offset, const float *__restrict__ src, int64_t ld_src,
                                   float *__restrict__ out, int64_t ld_out, int vec) {
    const int per = vec ? d / 4 : d;
    const int64_t total = n * per;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = t / per;
        const int f = (int)(t - i * per);
        const int64_t s = idx[i] + offset;
        if (vec)
            reinterpret_cast<float4 *>(out + i * ld_out)[f] =
                reinterpret_cast<const float4 *>(src + s * ld_src)[f];
        else
            out[i * ld_out + f] = src[s * ld_src + f];
    }
}

__global__ void scatter_add_rows_kernel(int64_t n, int d, const int64_t *__restrict__ idx,
                                        int64_t offset, const float *__restrict__ src,
                                        int64_t ld_src, float *__restrict__ dst, int64_t ld_dst) {
    const int64_t total = n * d;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = t / d;
        const int f = (int)(t - i * d);
        atomicAdd(dst + (idx[i] + offset) * ld_dst + f, src[i * ld_src + f]);
    }
}

__device__ __forceinline__ float softplus_f(float x) {
    // torch.nn.functional.softplus (beta 1, threshold 20)
    return x > 20.f ? x : log1pf(expf(x));
}

// One 16-lane group per sample at d = 64 (lanes stride the features by 4
// with float4 for d % 4 == 0; scalar otherwise).  Sums over d are reduced
// inside the group with xor shuffles, so d must be <= 4 * 64.  dw (the aux
// loss's feature weights) is summed over the workgroup's 16 samples in LDS
// first, then added with one global atomic per feature per workgroup (every
// sample adding to the same d floats would serialise on them).
template <int LPS>
__global__ __launch_bounds__(256) void bpr_kernel(
    int64_t batch, int d, const int64_t *__restrict__ users, const int64_t *__restrict__ pos,
    const int64_t *__restrict__ neg, int64_t off_u, int64_t off_i, const float *__restrict__ t,
    int64_t ld_t, const float *__restrict__ w, float *__restrict__ loss, float *__restrict__ l2,
    float g_loss, float g_l2, const float *__restrict__ g_loss_dev, const float *__restrict__ g_l2_dev,
    float *__restrict__ grad, int64_t ld_grad, float *__restrict__ dw) {
    constexpr int G = 64 / LPS;
    __shared__ float sdw[kBprMaxD];
    const int lane = threadIdx.x & 63;
    const int grp = lane / LPS;
    const int sub = lane - grp * LPS;
    const int64_t b = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * G + grp;
    const bool ok = b < batch;
    const int64_t ru = ok ? users[b] + off_u : 0;
    const int64_t rp = ok ? pos[b] + off_i : 0;
    const int64_t rn = ok ? neg[b] + off_i : 0;
    if (dw)
        for (int f = threadIdx.x; f < d; f += 256) sdw[f] = 0.f;
    float s = 0.f, q = 0.f;
    if (ok) {
        for (int f = sub; f < d; f += LPS) {
            const float u = t[ru * ld_t + f], p = t[rp * ld_t + f], n = t[rn * ld_t + f];
            const float wf = w ? w[f] : 1.f;
            // reference order: sum(u*n*w) - sum(u*p*w)  (trainer.py:538-539, 547-548)
            s += u * (n - p) * wf;
            q += u * u + p * p + n * n;
        }
    }
#pragma unroll
    for (int m = LPS >> 1; m >= 1; m >>= 1) {
        s += shfl_xor_f(s, m);
        q += shfl_xor_f(q, m);
    }
    if (ok && sub == 0) {
        if (loss) loss[b] = softplus_f(s);
        if (l2) l2[b] = q;
    }
    if (!grad && !dw) return;  // uniform over the grid
    if (dw) __syncthreads();   // sdw zeroed
    const float sig = 1.f / (1.f + expf(-s));  // d softplus(s) / ds
    const float gl = g_loss_dev ? g_loss * *g_loss_dev : g_loss;
    const float g2 = g_l2_dev ? g_l2 * *g_l2_dev : g_l2;
    const float cs = gl * sig, c2 = 2.f * g2;
    if (ok) {
        for (int f = sub; f < d; f += LPS) {
            const float u = t[ru * ld_t + f], p = t[rp * ld_t + f], n = t[rn * ld_t + f];
            const float wf = w ? w[f] : 1.f;
            if (grad) {
                atomicAdd(grad + ru * ld_grad + f, cs * (n - p) * wf + c2 * u);
                atomicAdd(grad + rp * ld_grad + f, -cs * u * wf + c2 * p);
                atomicAdd(grad + rn * ld_grad + f, cs * u * wf + c2 * n);
            }
            if (dw) atomicAdd(sdw + f, cs * u * (n - p));
        }
    }
    if (dw) {
        __syncthreads();
        for (int f = threadIdx.x; f < d; f += 256) atomicAdd(dw + f, sdw[f]);
    }
}

static unsigned grid_for(int64_t n, int block) {
    int64_t g = (n + block - 1) / block;
    if (g > 8192) g = 8192;
    return (unsigned)(g < 1 ? 1 : g);
}

}  // namespace igr

using namespace igr;

extern "C" int igr_gather_rows_f32(int64_t n, int32_t d, const int64_t *idx, int64_t offset,
                                   const float *src, int64_t ld_src, float *out, int64_t ld_out,
                                   void *stream) {
    return guarded("igr_gather_rows_f32", [&]() -> int {
        if (d <= 0 || ld_src < d || ld_out < d) return arg_error("igr_gather_rows_f32", "bad d / ld");
        if (n <= 0) return IGR_OK;
        const int vec = (d % 4 == 0 && ld_src % 4 == 0 && ld_out % 4 == 0 && aligned16(src) &&
                         aligned16(out));
        hipStream_t st = reinterpret_cast<hipStream_t>(stream);
        hipLaunchKernelGGL(gather_rows_kernel, dim3(grid_for(n * (vec ? d / 4 : d), 256)), dim3(256),
                           0, st, n, d, idx, offset, src, ld_src, out, ld_out, vec);
        return launch_status("igr_gather_rows_f32");
    });
}

extern "C" int igr_scatter_add_rows_f32(int64_t n, int32_t d, const int64_t *idx, int64_t offset,
                                        const float *src, int64_t ld_src, float *dst,
                                        int64_t ld_dst, void *stream) {
    return guarded("igr_scatter_add_rows_f32", [&]() -> int {
        if (d <= 0 || ld_src < d || ld_dst < d) return arg_error("igr_scatter_add_rows_f32", "bad d / ld");
        if (n <= 0) return IGR_OK;
        hipStream_t st = reinterpret_cast<hipStream_t>(stream);
        hipLaunchKernelGGL(scatter_add_rows_kernel, dim3(grid_for(n * d, 256)), dim3(256), 0, st, n,
                           d, idx, offset, src, ld_src, dst, ld_dst);
        return launch_status("igr_scatter_add_rows_f32");
    });
}

extern "C" int igr_bpr_fwd_bwd_f32(int64_t batch, int32_t d, const int64_t *users,
                                   const int64_t *pos, const int64_t *neg, int64_t off_u,
                                   int64_t off_i, const float *t, int64_t ld_t, const float *w,
                                   float *loss, float *l2, float g_loss, float g_l2,
                                   const float *g_loss_dev, const float *g_l2_dev, float *grad,
                                   int64_t ld_grad, float *dw, void *stream) {
    return guarded("igr_bpr_fwd_bwd_f32", [&]() -> int {
        if (d <= 0 || ld_t < d || (grad && ld_grad < d)) return arg_error("igr_bpr_fwd_bwd_f32", "bad d / ld");
        if (dw && d > kBprMaxD) return arg_error("igr_bpr_fwd_bwd_f32", "dw needs d <= 1024");
        if (batch <= 0) return IGR_OK;
        hipStream_t st = reinterpret_cast<hipStream_t>(stream);
        const int64_t per_block = 4 * (64 / 16);
        hipLaunchKernelGGL((bpr_kernel<16>), dim3((unsigned)((batch + per_block - 1) / per_block)),
                           dim3(256), 0, st, batch, d, users, pos, neg, off_u, off_i, t, ld_t, w,
                           loss, l2, g_loss, g_l2, g_loss_dev, g_l2_dev, grad, ld_grad, dw);
        return launch_status("igr_bpr_fwd_bwd_f32");
    });
}
