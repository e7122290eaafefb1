// att_shared.hip - the attention SDDMM with ONE source row serving every head (gfx950).
//
// AttIGCN (model.py:4257-4268) scores an edge (r <- c) per head as
//     alpha[e, h] = < x_q[r, h, :], x_k[c, h, :] >,   x_k[c, h, :] = W_k[h] E[c] + b_k[h],
// gathering the h * d floats of x_k[c] for every edge (1 KB at h = 4, d = 64).
// Since x_k is linear in E,
//     alpha[e, h] = < W_k[h]^T x_q[r, h, :], E[c] > + < x_q[r, h, :], b_k[h] >,
// and the second term is constant over the edges of row r, so the edge softmax
// that follows (model.py:4270-4274, a max-shifted softmax over each row) cancels
// it exactly.  With u[r, h, :] = W_k[h]^T x_q[r, h, :] folded into the query
// projection on the host side, every edge gathers only the d floats of E[c]:
// a quarter of the bytes at h = 4, and x_k is never formed.
//
//   igr_sddmm_shared_f32        out[eid, h] = < u[r, h, :], v[c, :] >
//   igr_spmm_shared_heads_f32   y[r, h, :]  = sum_{e in row r} rhs[eid, h] * x[c, :]
//                               (its gradient with respect to u)
// Both: one wave per destination row, d / 4 lanes per source row (one 16-byte load
// per lane), 64 / (d / 4) edges side by side, UE edges per lane group in flight.
#include "common.h"

namespace igr {

// Edges per lane group per trip.  Measured on MI355X (nnz 411 M, h = 4, d = 64):
// 1 -> 24.6 ms, 2 -> 26.9, 4 -> 46.8, 8 -> 134: the kernel is bound by the work its
// lanes do on a trip's empty slots (rows of ~20 edges fill few of a wide trip) and by
// registers, not by gathers in flight.
#ifndef IGR_SDDMM_SHARED_U
#define IGR_SDDMM_SHARED_U 1
#endif

constexpr int ilog2(int v) { return v <= 1 ? 0 : 1 + ilog2(v >> 1); }

template <int D, int H>
__global__ __launch_bounds__(256) void sddmm_shared_kernel(int64_t n_rows, const int64_t *__restrict__ row_ptr,
                                                           const int32_t *__restrict__ col,
                                                           const int64_t *__restrict__ eid,
                                                           const float *__restrict__ u, int64_t ld_u,
                                                           const float *__restrict__ v, int64_t ld_v,
                                                           float *__restrict__ out) {
    constexpr int LPE = D / 4;               // lanes per edge (source row)
    constexpr int EPW = 64 / LPE;            // edges side by side in a wave
    constexpr int UE = IGR_SDDMM_SHARED_U;   // edges per lane group per trip
    constexpr int TRIP = UE * EPW;           // edges per trip (divides 64)
    constexpr int V = UE * H;                // partial dots a lane holds: [edge][head]
    constexpr int RS = ilog2(V) < ilog2(LPE) ? ilog2(V) : ilog2(LPE);  // reduce-scatter steps
    constexpr int R = V >> RS;               // finished values per writer lane
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= n_rows) return;
    const int lane = threadIdx.x & 63;
    const int eg = lane / LPE;
    const int sub = lane - eg * LPE;
    float4 uq[H];
#pragma unroll
    for (int hh = 0; hh < H; ++hh) uq[hh] = *reinterpret_cast<const float4 *>(u + r * ld_u + hh * D + sub * 4);
    const float *vs = v + sub * 4;
    const int64_t b = row_ptr[r], e = row_ptr[r + 1];
    for (int64_t base = b; base < e; base += 64) {
        const int n = (int)min((int64_t)64, e - base);
        const int cl = lane < n ? col[base + lane] : 0;
        for (int t = 0; t < n; t += TRIP) {
            const int k0 = t + eg * UE;  // this group's first edge in the block
            float4 vk[UE];
#pragma unroll
            for (int j = 0; j < UE; ++j) {
                const int c = shfl_i(cl, (k0 + j) & 63);
                vk[j] = make_float4(0.f, 0.f, 0.f, 0.f);
                if (k0 + j < n) vk[j] = *reinterpret_cast<const float4 *>(vs + (int64_t)c * ld_v);
            }
            float sv[V];
#pragma unroll
            for (int j = 0; j < UE; ++j)
#pragma unroll
                for (int hh = 0; hh < H; ++hh)
                    sv[j * H + hh] = uq[hh].x * vk[j].x + uq[hh].y * vk[j].y + uq[hh].z * vk[j].z + uq[hh].w * vk[j].w;
            // butterfly reduce-scatter over the group's LPE lanes: at each step a lane keeps
            // one half of its values and adds the partner's copy of that half, so after RS
            // steps it holds R values summed over 2^RS lanes; value index = (top RS bits of
            // sub) * R + i
#pragma unroll
            for (int s = 0, cnt = V; s < RS; ++s, cnt >>= 1) {
                const int m = LPE >> (s + 1);
                const bool hi = (sub & m) != 0;
#pragma unroll
                for (int i = 0; i < cnt / 2; ++i) {
                    const float keep = hi ? sv[i + cnt / 2] : sv[i];
                    const float send = hi ? sv[i] : sv[i + cnt / 2];
                    sv[i] = keep + shfl_xor_f(send, m);
                }
            }
            // lanes left over (fewer values than lanes): plain xor steps
#pragma unroll
            for (int m = (LPE >> RS) >> 1; m >= 1; m >>= 1)
#pragma unroll
                for (int i = 0; i < R; ++i) sv[i] += shfl_xor_f(sv[i], m);
            if ((sub & ((LPE >> RS) - 1)) == 0) {
                const int first = (sub >> (ilog2(LPE) - RS)) * R;
#pragma unroll
                for (int i = 0; i < R; ++i) {
                    const int idx = first + i, j = idx / H, hh = idx - j * H;
                    const int k = k0 + j;
                    if (k < n) out[(eid ? eid[base + k] : base + k) * H + hh] = sv[i];
                }
            }
        }
    }
}

// y[r, hh, :] = sum over the edges of row r of rhs[eid, hh] * x[col, :]: each source row
// is gathered once and feeds H accumulators; the EPW lane groups take alternate edges
// and are summed in a fixed xor tree at the end (deterministic).
template <int D, int H>
__global__ __launch_bounds__(256) void spmm_shared_heads_kernel(int64_t n_rows, const int64_t *__restrict__ row_ptr,
                                                                const int32_t *__restrict__ col,
                                                                const int64_t *__restrict__ eid,
                                                                const float *__restrict__ x, int64_t ldx,
                                                                const float *__restrict__ rhs,
                                                                float *__restrict__ y, int64_t ldy) {
    constexpr int LPE = D / 4;
    constexpr int EPW = 64 / LPE;
    constexpr int UE = 4;
    constexpr int TRIP = UE * EPW;
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= n_rows) return;
    const int lane = threadIdx.x & 63;
    const int eg = lane / LPE;
    const int sub = lane - eg * LPE;
    const float *xs = x + sub * 4;
    float4 acc[H];
#pragma unroll
    for (int hh = 0; hh < H; ++hh) acc[hh] = make_float4(0.f, 0.f, 0.f, 0.f);
    const int64_t b = row_ptr[r], e = row_ptr[r + 1];
    for (int64_t base = b; base < e; base += 64) {
        const int n = (int)min((int64_t)64, e - base);
        const int cl = lane < n ? col[base + lane] : 0;
        const int64_t el = lane < n ? (eid ? eid[base + lane] : base + lane) : 0;
        for (int t = 0; t < n; t += TRIP) {
            const int k0 = t + eg * UE;
            float4 xv[UE];
            float wv[UE][H];
#pragma unroll
            for (int j = 0; j < UE; ++j) {
                const int src = (k0 + j) & 63;
                const int c = shfl_i(cl, src);
                const int64_t ee = ((int64_t)shfl_i((int)(el >> 32), src) << 32) | (uint32_t)shfl_i((int)el, src);
                xv[j] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
                for (int hh = 0; hh < H; ++hh) wv[j][hh] = 0.f;
                if (k0 + j < n) {
                    xv[j] = *reinterpret_cast<const float4 *>(xs + (int64_t)c * ldx);
#pragma unroll
                    for (int hh = 0; hh < H; ++hh) wv[j][hh] = rhs[ee * H + hh];
                }
            }
#pragma unroll
            for (int j = 0; j < UE; ++j)
#pragma unroll
                for (int hh = 0; hh < H; ++hh) acc[hh] = f4_fma(wv[j][hh], xv[j], acc[hh]);
        }
    }
#pragma unroll
    for (int m = LPE; m < 64; m <<= 1)
#pragma unroll
        for (int hh = 0; hh < H; ++hh) {
            acc[hh].x += shfl_xor_f(acc[hh].x, m);
            acc[hh].y += shfl_xor_f(acc[hh].y, m);
            acc[hh].z += shfl_xor_f(acc[hh].z, m);
            acc[hh].w += shfl_xor_f(acc[hh].w, m);
        }
    if (eg == 0) {
#pragma unroll
        for (int hh = 0; hh < H; ++hh) *reinterpret_cast<float4 *>(y + r * ldy + hh * D + sub * 4) = acc[hh];
    }
}

template <template <int, int> class Launch, class... Args>
static bool dispatch_dh(int d, int h, Args... args) {
#define IGR_DH(DD, HH) if (d == DD && h == HH) { Launch<DD, HH>::go(args...); return true; }
    IGR_DH(32, 1) IGR_DH(32, 2) IGR_DH(32, 4) IGR_DH(32, 8)
    IGR_DH(64, 1) IGR_DH(64, 2) IGR_DH(64, 4) IGR_DH(64, 8)
    IGR_DH(128, 1) IGR_DH(128, 2) IGR_DH(128, 4)
    IGR_DH(256, 1) IGR_DH(256, 2)
#undef IGR_DH
    return false;
}

template <int D, int H>
struct LaunchSddmmShared {
    static void go(const igr_csr *g, const float *u, int64_t ld_u, const float *v, int64_t ld_v, float *out,
                   hipStream_t st) {
        hipLaunchKernelGGL((sddmm_shared_kernel<D, H>), dim3((unsigned)((g->n_rows + 3) / 4)), dim3(256), 0, st,
                           g->n_rows, g->row_ptr, g->col_idx, g->edge_id, u, ld_u, v, ld_v, out);
    }
};

template <int D, int H>
struct LaunchSpmmShared {
    static void go(const igr_csr *g, const float *x, int64_t ldx, const float *rhs, float *y, int64_t ldy,
                   hipStream_t st) {
        hipLaunchKernelGGL((spmm_shared_heads_kernel<D, H>), dim3((unsigned)((g->n_rows + 3) / 4)), dim3(256), 0, st,
                           g->n_rows, g->row_ptr, g->col_idx, g->edge_id, x, ldx, rhs, y, ldy);
    }
};

}  // namespace igr

using namespace igr;

extern "C" int igr_sddmm_shared_f32(const igr_csr *g, int32_t h, int32_t d, const float *u, int64_t ld_u,
                                    const float *v, int64_t ld_v, float *out, void *stream) {
    return guarded("igr_sddmm_shared_f32", [&]() -> int {
        const char *fn = "igr_sddmm_shared_f32";
        if (!g || h <= 0 || d <= 0) return arg_error(fn, "bad graph / h / d");
        if (ld_u < (int64_t)h * d || ld_v < d) return arg_error(fn, "leading dimension too small");
        if (g->n_rows == 0 || g->nnz == 0) return IGR_OK;
        if (!u || !v || !out) return arg_error(fn, "NULL pointer");
        if (ld_u % 4 || ld_v % 4 || !aligned16(u) || !aligned16(v))
            return arg_error(fn, "u / v must be 16-byte aligned with leading dimensions a multiple of 4");
        if (!dispatch_dh<LaunchSddmmShared>(d, h, g, u, ld_u, v, ld_v, out, reinterpret_cast<hipStream_t>(stream)))
            return arg_error(fn, "supported: d in {32, 64, 128, 256} with h * d <= 512, h a power of two");
        return launch_status(fn);
    });
}

extern "C" int igr_spmm_shared_heads_f32(const igr_csr *g, int32_t h, int32_t d, const float *x, int64_t ldx,
                                         const float *rhs, float *y, int64_t ldy, void *stream) {
    return guarded("igr_spmm_shared_heads_f32", [&]() -> int {
        const char *fn = "igr_spmm_shared_heads_f32";
        if (!g || h <= 0 || d <= 0) return arg_error(fn, "bad graph / h / d");
        if (ldx < d || ldy < (int64_t)h * d) return arg_error(fn, "leading dimension too small");
        if (g->n_rows == 0) return IGR_OK;
        if (!y || (g->nnz > 0 && (!x || !rhs))) return arg_error(fn, "NULL pointer");
        if (ldx % 4 || ldy % 4 || !aligned16(x) || !aligned16(y))
            return arg_error(fn, "x / y must be 16-byte aligned with leading dimensions a multiple of 4");
        if (!dispatch_dh<LaunchSpmmShared>(d, h, g, x, ldx, rhs, y, ldy, reinterpret_cast<hipStream_t>(stream)))
            return arg_error(fn, "supported: d in {32, 64, 128, 256} with h * d <= 512, h a power of two");
        return launch_status(fn);
    });
}
