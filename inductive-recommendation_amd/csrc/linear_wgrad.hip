// linear_wgrad.hip - weight and bias gradients of a Linear over every node (gfx950).
//
//   dW[n, c] = sum_m dy[m, n] * x[m, c],   db[n] = sum_m dy[m, n]
//
// for y = x W^T + b with M = node count rows, k_in in {32, 64, 128} input columns and
// n_out a multiple of 64 (NGCF's Linear(d, d), model.py:4039, and AttIGCN's
// Linear(d, 4d), model.py:4259, 4264 - the backward of loss.backward(), trainer.py:553).
// As a GEMM this is a few output tiles with K = node count; here it is a stream:
//  * a wave owns 64 output rows n and every n_ranges-th group of data rows m, and keeps
//    its 64 x k_in block of dW in MFMA accumulators for the whole launch;
//  * dy and x go from global memory straight into MFMA operands - no LDS, no barrier:
//    lane (i, kk) loads the 16 bytes dy[m + kk][n0 + 4 i .. 4 i + 3], which are the A
//    operands of FOUR 16x16x4 MFMAs whose output row i stands for n0 + 4 i + t
//    (t = 0..3), and likewise 16 bytes of x[m + kk] as the B operands of four column
//    tiles (column 4 j + u); so every load instruction moves whole 256-byte row
//    segments and one pair of loads feeds 16 MFMAs;
//  * the bias gradient falls out of the same dy registers (a running sum per lane,
//    folded over the four kk lane groups at the end);
//  * every wave writes its partial block to a workspace and a second kernel adds the
//    partials in range order: the same bits on every run.
// The 4 waves of a workgroup take the n blocks of the SAME groups (n_out = 256), so the
// x rows they all read arrive once from L2.
#include <algorithm>
#include <type_traits>

#include "common.h"

namespace igr {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// Measured on MI355X, Linear(64, 256) on 1.1 M rows (k steps per load group x waves in all):
// 8 x 1024 -> 352-356 us, 12 x 1024 -> 352, 16 x 1024 -> 382, 4 x 1024 -> 385, 4 x 2048 -> 414-442,
// 6 x 2048 -> 395-474, 2 x 2048 at 4 waves per SIMD -> 426, 4 x 4096 -> 595, 16 x 512 -> 635:
// one wave per SIMD with a deep prefetch wins (fewer partial blocks to write and add, and
// every wave's MFMAs run from registers that were loaded two groups ago).
#ifndef IGR_WGRAD_PF
#define IGR_WGRAD_PF 8
#endif
#ifndef IGR_WGRAD_OCC
#define IGR_WGRAD_OCC 1   // workgroups per CU the register budget allows
#endif
#ifndef IGR_WGRAD_WAVES
#define IGR_WGRAD_WAVES 1024  // waves in all: one per SIMD
#endif
constexpr int WG_PF = IGR_WGRAD_PF;  // k steps (of 4 data rows) whose loads are issued before their MFMAs

// NT = k_in / 16 column tiles (8: two float4 of x per lane, 4: float4, 2: float2)
template <int NT>
__global__ __launch_bounds__(256, IGR_WGRAD_OCC) void linear_wgrad_kernel(int64_t M, int n_out, int nb_in_wg,
                                                           const float *__restrict__ dy, int64_t ld_dy,
                                                           const float *__restrict__ x, int64_t ld_x,
                                                           int64_t n_ranges, float *__restrict__ part,
                                                           float *__restrict__ part_b) {
    constexpr int KIN = 16 * NT;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int i16 = lane & 15, kk = lane >> 4;
    const int ranges_in_wg = 4 / nb_in_wg;
    const int64_t range = (int64_t)blockIdx.x * ranges_in_wg + wave / nb_in_wg;
    const int nb = blockIdx.y * nb_in_wg + wave % nb_in_wg;
    if (range >= n_ranges) return;
    const int n0 = nb * 64;
    const float *dyp = dy + n0 + 4 * i16;
    const float *xp = x + NT * i16;
    f32x4 acc[4][NT];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int u = 0; u < NT; ++u) acc[t][u] = f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 bsum = f32x4{0.f, 0.f, 0.f, 0.f};

    // one group = WG_PF k steps of 4 data rows; a lane's loads of a group: WG_PF x (16 bytes
    // of dy + 4 NT bytes of x).  Groups are dealt to the workers round-robin (worker w takes
    // groups w, w + n_ranges, ...), so at any moment the whole chip reads one window of
    // consecutive rows, as a streaming copy does (measured equal to one contiguous range
    // per worker; kept because it needs no per-range tail).
    constexpr int64_t GR = 4 * WG_PF;  // data rows per group
    const int64_t n_full = M / GR;     // whole groups
    auto load_group = [&](f32x4 (&a)[WG_PF], float (&b)[WG_PF][NT], int64_t g, auto clamp)
                          __attribute__((always_inline)) {
        constexpr bool CLAMP = decltype(clamp)::value;
        // a whole group past the last one (a prefetch that will not be used) reads the last whole group
        const int64_t gb = (CLAMP || g < n_full ? g : n_full - 1) * GR;
#pragma unroll
        for (int s = 0; s < WG_PF; ++s) {
            const int64_t m = gb + 4 * s + kk;
            const int64_t mc = (!CLAMP || m < M) ? m : M - 1;
            a[s] = *reinterpret_cast<const f32x4 *>(dyp + mc * ld_dy);
            if (NT == 8) {
                const f32x4 v0 = *reinterpret_cast<const f32x4 *>(xp + mc * ld_x);
                const f32x4 v1 = *reinterpret_cast<const f32x4 *>(xp + mc * ld_x + 4);
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    b[s][u] = v0[u];
                    b[s][4 + u] = v1[u];
                }
            } else if (NT == 4) {
                const f32x4 v = *reinterpret_cast<const f32x4 *>(xp + mc * ld_x);
#pragma unroll
                for (int u = 0; u < NT; ++u) b[s][u] = v[u];
            } else {
                const f32x2 v = *reinterpret_cast<const f32x2 *>(xp + mc * ld_x);
#pragma unroll
                for (int u = 0; u < NT; ++u) b[s][u] = v[u];
            }
        }
    };
    // after every load of the group has been issued: rows past the matrix count as zeros
    auto mask_group = [&](f32x4 (&a)[WG_PF], float (&b)[WG_PF][NT], int64_t g) __attribute__((always_inline)) {
#pragma unroll
        for (int s = 0; s < WG_PF; ++s) {
            const bool valid = g * GR + 4 * s + kk < M;
#pragma unroll
            for (int t = 0; t < 4; ++t) a[s][t] = valid ? a[s][t] : 0.f;
#pragma unroll
            for (int u = 0; u < NT; ++u) b[s][u] = valid ? b[s][u] : 0.f;
        }
    };
    auto fma_group = [&](const f32x4 (&a)[WG_PF], const float (&b)[WG_PF][NT]) __attribute__((always_inline)) {
#pragma unroll
        for (int s = 0; s < WG_PF; ++s) {
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int u = 0; u < NT; ++u)
                    acc[t][u] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s][t], b[s][u], acc[t][u], 0, 0, 0);
            bsum += a[s];
        }
    };
    f32x4 a0[WG_PF], a1[WG_PF];
    float b0[WG_PF][NT], b1[WG_PF][NT];
    // whole groups, double-buffered: the next group's loads are in flight under this group's
    // MFMAs (scheduling barriers keep each group's loads together and ahead of the other
    // group's MFMAs: left alone, the scheduler sinks every load next to its first use)
    int64_t g = range;
    if (g < n_full) load_group(a0, b0, g, std::false_type{});
    while (g < n_full) {
        load_group(a1, b1, g + n_ranges, std::false_type{});
        __builtin_amdgcn_sched_barrier(0);
        fma_group(a0, b0);
        __builtin_amdgcn_sched_barrier(0);
        g += n_ranges;
        if (g >= n_full) break;
        load_group(a0, b0, g + n_ranges, std::false_type{});
        __builtin_amdgcn_sched_barrier(0);
        fma_group(a1, b1);
        __builtin_amdgcn_sched_barrier(0);
        g += n_ranges;
    }
    // the ragged last group (rows n_full GR .. M - 1) goes to the worker whose turn it is
    if (n_full * GR < M && n_full % n_ranges == range) {
        load_group(a0, b0, n_full, std::true_type{});
        __builtin_amdgcn_sched_barrier(0);
        mask_group(a0, b0, n_full);
        fma_group(a0, b0);
    }
    // D of tile (t, u): lane holds rows 4 kk + r (r = 0..3) of column i16, i.e.
    // n = n0 + 4 (4 kk + r) + t and input columns NT i16 + u: NT consecutive floats
    float *pw = part + (range * n_out + n0) * KIN;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float *o = pw + (int64_t)(4 * (4 * kk + r) + t) * KIN + NT * i16;
            if (NT == 8) {
                *reinterpret_cast<f32x4 *>(o) = f32x4{acc[t][0][r], acc[t][1][r], acc[t][2][r], acc[t][3][r]};
                *reinterpret_cast<f32x4 *>(o + 4) =
                    f32x4{acc[t][NT - 4][r], acc[t][NT - 3][r], acc[t][NT - 2][r], acc[t][NT - 1][r]};
            } else if (NT == 4)
                *reinterpret_cast<f32x4 *>(o) = f32x4{acc[t][0][r], acc[t][1][r], acc[t][2][r], acc[t][3][r]};
            else
                *reinterpret_cast<f32x2 *>(o) = f32x2{acc[t][0][r], acc[t][NT - 1][r]};
        }
    if (part_b) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            bsum[q] += shfl_xor_f(bsum[q], 16);
            bsum[q] += shfl_xor_f(bsum[q], 32);
        }
        if (kk == 0) *reinterpret_cast<f32x4 *>(part_b + range * n_out + n0 + 4 * i16) = bsum;
    }
}

// dw[i] = sum_p part[p * nw + i] (i < nw) and db[j] = sum_p part_b[p * nb + j] (j < nb): 16
// lanes per element, lane l adds partials l, l + 16, ... in order and the 16 lane sums are
// added in a fixed xor tree - the same bits on every run.  (One thread per element walked
// the workers serially: 12 us of dependent loads for 152 workers.)
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(int64_t nw, int64_t nb, int64_t P,
                                                           const float *__restrict__ part,
                                                           const float *__restrict__ part_b, float *__restrict__ dw,
                                                           int64_t ld_dw, int cols, float *__restrict__ db) {
    const int l = threadIdx.x & 15;
    int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4;
    if (i >= nw + nb) return;  // whole 16-lane groups leave together
    const bool bias = i >= nw;
    const float *src = bias ? part_b : part;
    const int64_t n = bias ? nb : nw;
    if (bias) i -= nw;
    float s0 = 0.f, s1 = 0.f;
    int64_t p = l;
    for (; p + 16 < P; p += 32) {
        s0 += src[p * n + i];
        s1 += src[(p + 16) * n + i];
    }
    if (p < P) s0 += src[p * n + i];
    float v = s0 + s1;
    v += shfl_xor_f(v, 8);
    v += shfl_xor_f(v, 4);
    v += shfl_xor_f(v, 2);
    v += shfl_xor_f(v, 1);
    if (l != 0) return;
    if (bias) {
        db[i] = v;
    } else {
        const int64_t r = i / cols;
        dw[r * ld_dw + (i - r * cols)] = v;
    }
}

// workers per 64-row block of dW: about IGR_WGRAD_WAVES waves in all, at least 64 data rows each
static int64_t wgrad_ranges(int64_t m, int32_t n_out) {
    const int64_t target = std::max<int64_t>(1, IGR_WGRAD_WAVES / (n_out / 64));
    return std::max<int64_t>(1, std::min<int64_t>(target, m / 64));
}

static bool wgrad_shape_ok(int64_t m, int32_t n_out, int32_t k_in) {
    const int nb = n_out / 64;
    return m > 0 && n_out > 0 && n_out % 64 == 0 && (k_in == 32 || k_in == 64 || k_in == 128) &&
           (nb == 1 || nb == 2 || nb % 4 == 0);
}

}  // namespace igr

using namespace igr;

extern "C" int64_t igr_linear_wgrad_workspace_size(int64_t m, int32_t n_out, int32_t k_in) {
    if (!wgrad_shape_ok(m, n_out, k_in)) return 0;
    return wgrad_ranges(m, n_out) * (int64_t)n_out * (k_in + 1) * (int64_t)sizeof(float);
}

extern "C" int igr_linear_wgrad_f32(int64_t m, int32_t n_out, int32_t k_in, const float *dy, int64_t ld_dy,
                                    const float *x, int64_t ld_x, float *dw, int64_t ld_dw, float *db,
                                    void *workspace, int64_t ws_bytes, void *stream) {
    return guarded("igr_linear_wgrad_f32", [&]() -> int {
        const char *fn = "igr_linear_wgrad_f32";
        if (!wgrad_shape_ok(m, n_out, k_in))
            return arg_error(fn, "supported: k_in in {32, 64, 128}, n_out in {64, 128} or a multiple of 256, m > 0");
        if (!dy || !x || !dw) return arg_error(fn, "NULL pointer");
        if (ld_dy < n_out || ld_x < k_in || ld_dw < k_in) return arg_error(fn, "leading dimension too small");
        if (ld_dy % 4 || ld_x % 4 || !aligned16(dy) || !aligned16(x))
            return arg_error(fn, "dy / x must be 16-byte aligned with leading dimensions a multiple of 4");
        const int64_t need = igr_linear_wgrad_workspace_size(m, n_out, k_in);
        if (!workspace || ws_bytes < need || !aligned16(workspace))
            return arg_error(fn, "workspace of igr_linear_wgrad_workspace_size(m, n_out, k_in) bytes (16-byte aligned) needed");
        hipStream_t st = reinterpret_cast<hipStream_t>(stream);
        const int64_t ranges = wgrad_ranges(m, n_out);
        const int nb = n_out / 64;
        const int nb_in_wg = nb < 4 ? nb : 4;
        const int ranges_in_wg = 4 / nb_in_wg;
        float *part = static_cast<float *>(workspace);
        float *part_b = db ? part + ranges * (int64_t)n_out * k_in : nullptr;
        const dim3 grid((unsigned)((ranges + ranges_in_wg - 1) / ranges_in_wg), (unsigned)(nb / nb_in_wg));
        if (k_in == 128)
            hipLaunchKernelGGL((linear_wgrad_kernel<8>), grid, dim3(256), 0, st, m, (int)n_out, nb_in_wg, dy, ld_dy, x,
                               ld_x, ranges, part, part_b);
        else if (k_in == 64)
            hipLaunchKernelGGL((linear_wgrad_kernel<4>), grid, dim3(256), 0, st, m, (int)n_out, nb_in_wg, dy, ld_dy, x,
                               ld_x, ranges, part, part_b);
        else
            hipLaunchKernelGGL((linear_wgrad_kernel<2>), grid, dim3(256), 0, st, m, (int)n_out, nb_in_wg, dy, ld_dy, x,
                               ld_x, ranges, part, part_b);
        const int64_t nw = (int64_t)n_out * k_in, nbias = db ? n_out : 0;
        hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((nw + nbias + 15) / 16)), dim3(256), 0, st, nw, nbias,
                           ranges, part, part_b, dw, ld_dw, (int)k_in, db);
        return launch_status(fn);
    });
}
