// bpr.hip - BPR negative-sample embedding gathers and the fused BPR loss
// (gfx950).
//
//   igr_gather_rows_f32       rep[users], rep[n_users + pos/neg]   model.py:4048-4049
//   igr_bpr_fwd_bwd_f32       NGCF.bpr_forward + IGCNTrainer loss   model.py:4046-4052,
//                             (BPR term and the aux term with w)    trainer.py:536-549
// The gathers' backward (index_put accumulate) is in rowsort.hip.  The fused
// BPR gradient adds each table row's terms in a fixed order as well (no float
// atomics): the rows a batch touches arrive sorted (igr_rowsort), one thread
// per distinct row and 4-float chunk walks that row's samples in order.
#include "common.h"
#include "segsum.h"

namespace igr {

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

__device__ __forceinline__ float softplus_f(float x) {
    // torch.nn.functional.softplus (beta 1, threshold 20)
    return x > 20.f ? x : log1pf(expf(x));
}

// One 16-lane group per sample (lanes stride the features).  Sums over d are
// reduced inside the group with xor shuffles.  Forward: loss / l2 per sample.
// Backward (terms / grad / dw_part given), with cs = g_loss * sigmoid(s_b):
//   terms   [3 * batch, d]: the gradient term of entry e = role * batch + b
//           (role 0 users, 1 pos, 2 neg) - summed per table row afterwards, in
//           entry order, by seg_scatter_add_kernel over the sorted rows;
//   grad    instead of terms when the 3 * batch rows are distinct by contract:
//           every entry adds its own term in place;
//   dw_part [blocks, d]: the workgroup's 16 samples' dw terms summed in sample
//           order (LDS stage, no atomics).
template <int LPS>
__global__ __launch_bounds__(256) void bpr_kernel(
    int64_t batch, int d, const int64_t *__restrict__ users, const int64_t *__restrict__ pos,
    const int64_t *__restrict__ neg, int64_t off_u, int64_t off_i, const float *__restrict__ t,
    int64_t ld_t, const float *__restrict__ w, float *__restrict__ loss, float *__restrict__ l2,
    float g_loss, float g_l2, const float *__restrict__ g_loss_dev, const float *__restrict__ g_l2_dev,
    float *__restrict__ terms, float *__restrict__ grad, int64_t ld_grad, float *__restrict__ dw_part) {
    constexpr int G = 64 / LPS;
    constexpr int SPB = 4 * G;   // samples per workgroup
    constexpr int FB = 256;      // features staged per round
    __shared__ float stage[SPB][FB];
    const int lane = threadIdx.x & 63;
    const int grp = lane / LPS;
    const int sub = lane - grp * LPS;
    const int sib = (threadIdx.x >> 6) * G + grp;  // sample within the workgroup
    const int64_t b = (int64_t)blockIdx.x * SPB + sib;
    const bool ok = b < batch;
    const int64_t ru = ok ? users[b] + off_u : 0;
    const int64_t rp = ok ? pos[b] + off_i : 0;
    const int64_t rn = ok ? neg[b] + off_i : 0;
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
    if (!terms && !grad && !dw_part) return;  // uniform over the grid
    const float sig = 1.f / (1.f + expf(-s));  // d softplus(s) / ds
    const float cs = (g_loss_dev ? g_loss * *g_loss_dev : g_loss) * sig;
    const float c2 = 2.f * (g_l2_dev ? g_l2 * *g_l2_dev : g_l2);
    if (ok && (terms || grad)) {
        for (int f = sub; f < d; f += LPS) {
            const float u = t[ru * ld_t + f], p = t[rp * ld_t + f], n = t[rn * ld_t + f];
            const float wf = w ? w[f] : 1.f;
            // gradient of softplus(sum_f u (n - p) w) and of |u|^2 + |p|^2 + |n|^2
            const float tu = fmaf(c2, u, cs * (n - p) * wf);
            const float tp = fmaf(c2, p, -cs * u * wf);
            const float tn = fmaf(c2, n, cs * u * wf);
            if (terms) {
                terms[b * d + f] = tu;
                terms[(batch + b) * d + f] = tp;
                terms[(2 * batch + b) * d + f] = tn;
            } else {
                grad[ru * ld_grad + f] += tu;
                grad[rp * ld_grad + f] += tp;
                grad[rn * ld_grad + f] += tn;
            }
        }
    }
    if (!dw_part) return;
    for (int f0 = 0; f0 < d; f0 += FB) {
        for (int f = f0 + sub; f < min(d, f0 + FB); f += LPS) {
            float v = 0.f;
            if (ok) {
                const float u = t[ru * ld_t + f], p = t[rp * ld_t + f], n = t[rn * ld_t + f];
                v = cs * u * (n - p);
            }
            stage[sib][f - f0] = v;
        }
        __syncthreads();
        for (int f = f0 + threadIdx.x; f < min(d, f0 + FB); f += 256) {
            float a = 0.f;
#pragma unroll
            for (int k = 0; k < SPB; ++k) a += stage[k][f - f0];
            dw_part[(int64_t)blockIdx.x * d + f] = a;
        }
        __syncthreads();
    }
}

// Backward, second launch.  Workgroups [0, grad_blocks): the gradient rows -
// seg_scatter_add over the sorted rows (one thread per sorted position and
// feature chunk; a row's first position adds the row's terms in entry order).
// The remaining workgroups: dw[f] += sum_j dw_part[j][f] for 64 features each,
// the partials added in workgroup order (four strided chains per feature,
// combined in a fixed tree through LDS).
template <class V>
__global__ __launch_bounds__(256) void bpr_finish_kernel(int64_t n, int per, const uint64_t *__restrict__ keys,
                                                         const float *__restrict__ terms, int64_t ld_terms,
                                                         float *__restrict__ grad, int64_t ld_grad,
                                                         int64_t grad_blocks, int d,
                                                         const float *__restrict__ dw_part, int64_t n_part,
                                                         float *__restrict__ dw) {
    __shared__ float red[4][64];
    if ((int64_t)blockIdx.x >= grad_blocks) {
        const int f = (int)(((int64_t)blockIdx.x - grad_blocks) * 64) + (threadIdx.x & 63);
        const int c = threadIdx.x >> 6;
        float a0 = 0.f, a1 = 0.f;
        if (f < d) {
            int64_t j = c;
            for (; j + 4 < n_part; j += 8) {
                a0 += dw_part[j * d + f];
                a1 += dw_part[(j + 4) * d + f];
            }
            if (j < n_part) a0 += dw_part[j * d + f];
        }
        red[c][threadIdx.x & 63] = a0 + a1;
        __syncthreads();
        if (c == 0 && f < d) dw[f] += (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
        return;
    }
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= n * per) return;
    const int64_t k = t / per;
    const int f = (int)(t - k * per);
    const uint64_t row = keys[k] >> 32;
    if (k > 0 && (keys[k - 1] >> 32) == row) return;
    float *o = grad + (int64_t)row * ld_grad;
    V::store(o, f, seg_run_sum<V, false>(V::load(o, f), n, k, row, keys, terms, ld_terms, f, 1.f));
}

// out[0] = mean(a), out[1] = mean(b) (b nullable) of n per-sample values, one
// workgroup, every sum in a fixed order: thread t adds elements t, t + 1024, ...
// in order, then a fixed tree over the 1024 partials.
__global__ __launch_bounds__(1024) void means_kernel(int64_t n, const float *__restrict__ a,
                                                     const float *__restrict__ b, float *__restrict__ out) {
    __shared__ float red[2][1024];
    const int t = threadIdx.x;
    float sa = 0.f, sb = 0.f;
    for (int64_t i = t; i < n; i += 1024) {
        sa += a[i];
        if (b) sb += b[i];
    }
    red[0][t] = sa;
    red[1][t] = sb;
    __syncthreads();
    for (int s = 512; s > 0; s >>= 1) {
        if (t < s) {
            red[0][t] += red[0][t + s];
            red[1][t] += red[1][t + s];
        }
        __syncthreads();
    }
    if (t == 0) {
        out[0] = red[0][0] / (float)n;
        if (b) out[1] = red[1][0] / (float)n;
    }
}

// reg = c_l2 * l2 + c_aux * aux; loss = bpr + reg (trainer.py:551-552, 424-425),
// every operation rounded on its own as in the scalar tensor expression, and
// *loss_sum += loss * weight for the epoch's running sum.
__global__ void loss_combine_kernel(const float *__restrict__ bpr, const float *__restrict__ l2,
                                    const float *__restrict__ aux, float c_l2, float c_aux, float weight,
                                    float *__restrict__ loss, float *__restrict__ loss_sum) {
    // no contraction into fma: each product and sum is rounded as the tensor ops round them
#pragma clang fp contract(off)
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    float reg = l2 ? c_l2 * *l2 : 0.f;
    if (aux) {
        const float a = c_aux * *aux;
        reg = l2 ? reg + a : a;
    }
    const float v = (l2 || aux) ? *bpr + reg : *bpr;
    *loss = v;
    if (loss_sum) {
        const float add = v * weight;
        *loss_sum = *loss_sum + add;
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

extern "C" int64_t igr_bpr_workspace_floats(int64_t batch, int32_t d) {
    if (batch <= 0 || d <= 0) return 0;
    return 3 * batch * (int64_t)d + ((batch + 15) / 16) * (int64_t)d;
}

extern "C" int igr_bpr_fwd_bwd_f32(int64_t batch, int32_t d, const int64_t *users,
                                   const int64_t *pos, const int64_t *neg, int64_t off_u,
                                   int64_t off_i, const float *t, int64_t ld_t, const float *w,
                                   float *loss, float *l2, float g_loss, float g_l2,
                                   const float *g_loss_dev, const float *g_l2_dev, float *grad,
                                   int64_t ld_grad, float *dw, const uint64_t *sorted, float *workspace,
                                   void *stream) {
    return guarded("igr_bpr_fwd_bwd_f32", [&]() -> int {
        const char *fn = "igr_bpr_fwd_bwd_f32";
        if (d <= 0 || ld_t < d || (grad && ld_grad < d)) return arg_error(fn, "bad d / ld");
        if (batch <= 0) return IGR_OK;
        if (batch > 2147483647 / 3) return arg_error(fn, "batch too large");
        if (((grad && sorted) || dw) && !workspace)
            return arg_error(fn, "the backward needs a workspace of igr_bpr_workspace_floats(batch, d) floats");
        hipStream_t st = reinterpret_cast<hipStream_t>(stream);
        constexpr int64_t per_block = 4 * (64 / 16);
        const int64_t blocks = (batch + per_block - 1) / per_block;
        float *terms = (grad && sorted) ? workspace : nullptr;
        float *dw_part = dw ? workspace + 3 * batch * (int64_t)d : nullptr;
        hipLaunchKernelGGL((bpr_kernel<16>), dim3((unsigned)blocks), dim3(256), 0, st, batch, d, users, pos, neg,
                           off_u, off_i, t, ld_t, w, loss, l2, g_loss, g_l2, g_loss_dev, g_l2_dev, terms,
                           (grad && !sorted) ? grad : nullptr, ld_grad, dw_part);
        if (terms || dw) {
            const int64_t n = terms ? 3 * batch : 0;
            const bool vec = d % 4 == 0 && ld_grad % 4 == 0 && aligned16(workspace) && aligned16(grad);
            const int per = vec ? d / 4 : d;
            const int64_t grad_blocks = (n * per + 255) / 256;
            const int64_t dw_blocks = dw ? (d + 63) / 64 : 0;
            const dim3 grid((unsigned)(grad_blocks + dw_blocks));
            if (vec)
                hipLaunchKernelGGL((bpr_finish_kernel<SegAdd4>), grid, dim3(256), 0, st, n, per, sorted, terms,
                                   (int64_t)d, grad, ld_grad, grad_blocks, (int)d, dw_part, blocks, dw);
            else
                hipLaunchKernelGGL((bpr_finish_kernel<SegAdd1>), grid, dim3(256), 0, st, n, per, sorted, terms,
                                   (int64_t)d, grad, ld_grad, grad_blocks, (int)d, dw_part, blocks, dw);
        }
        return launch_status(fn);
    });
}

extern "C" int igr_means_f32(int64_t n, const float *a, const float *b, float *out, void *stream) {
    return guarded("igr_means_f32", [&]() -> int {
        if (n <= 0 || !a || !out) return arg_error("igr_means_f32", "n <= 0 or a null pointer");
        hipLaunchKernelGGL(means_kernel, dim3(1), dim3(1024), 0, reinterpret_cast<hipStream_t>(stream), n, a, b, out);
        return launch_status("igr_means_f32");
    });
}

extern "C" int igr_loss_combine_f32(const float *bpr, const float *l2, const float *aux, float c_l2, float c_aux,
                                    float weight, float *loss, float *loss_sum, void *stream) {
    return guarded("igr_loss_combine_f32", [&]() -> int {
        if (!bpr || !loss) return arg_error("igr_loss_combine_f32", "bpr and loss must be given");
        hipLaunchKernelGGL(loss_combine_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), bpr, l2,
                           aux, c_l2, c_aux, weight, loss, loss_sum);
        return launch_status("igr_loss_combine_f32");
    });
}
