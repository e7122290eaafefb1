// gemm.hip - fp32 GEMM on gfx950 matrix cores (v_mfma_f32_16x16x4_f32).
//
// The dense projections on the GCN path: NGCF gc/bi layers Linear(d, d)
// (model.py:3998-4004, 4039) and AttIGCN weight_q / weight_k Linear(d, 4d)
// (model.py:4242-4243, 4259, 4264), forward and backward.  Shapes are tall and
// skinny (M = node count, N, K = d..4d), so one 64x64 output tile per
// workgroup, K staged through LDS 16 at a time.  The weight gradients
// (M, N = d..4d, K = node count) have only a few output tiles: there K is
// split over workgroups (grid.z) into a workspace and summed in split order.  f32-input MFMA is an exact
// k-ordered fmaf chain (no xf32 on gfx950), i.e. fp32 semantics.
#include "common.h"

namespace igr {

typedef float f32x4 __attribute__((ext_vector_type(4)));

#ifndef IGR_GEMM_BK
#define IGR_GEMM_BK 16
#endif
constexpr int BM = 64, BN = 64, BK = IGR_GEMM_BK;
constexpr int LPT = BM * BK / 256;  // elements of each operand tile one thread stages

// One 64x64 output tile per workgroup (2x2 waves of 32x32, 2x2 MFMA 16x16x4 each).
// K moves through double-buffered LDS tiles of BK; the next tile's global loads
// are issued before the current tile's MFMAs, so their latency hides under the
// math (one barrier per K step: a buffer is rewritten only after every wave has
// passed the barrier that follows its last read).
template <bool TA, bool TB>
__global__ __launch_bounds__(256) void gemm_f32_mfma(int64_t M, int64_t N, int64_t K,
                                                     const float *__restrict__ A, int64_t lda,
                                                     const float *__restrict__ B, int64_t ldb,
                                                     const float *__restrict__ bias,
                                                     float *__restrict__ C, int64_t ldc, int64_t kc,
                                                     int64_t zstride) {
    // split-K: this workgroup takes K range [z kc, min(K, (z+1) kc)) and writes
    // its partial tile to C + z * zstride (kc = K, zstride = 0 without a split)
    const int64_t k_lo = (int64_t)blockIdx.z * kc;
    const int64_t k_hi = k_lo + kc < K ? k_lo + kc : K;
    C += (int64_t)blockIdx.z * zstride;
    // LDS images [k][m] and [k][n], padded by one float to break bank strides.
    __shared__ float As[2][BK][BM + 1];
    __shared__ float Bs[2][BK][BN + 1];
    const int t = threadIdx.x;
    const int lane = t & 63, wave = t >> 6;
    const int wm = wave >> 1, wn = wave & 1;  // 2x2 waves, 32x32 each
    const int64_t m0 = (int64_t)blockIdx.x * BM, n0 = (int64_t)blockIdx.y * BN;
    f32x4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // staging coordinates of element i of this thread (same for every K step)
    auto a_mk = [&](int i, int &mm, int &kk) {
        const int idx = t + i * 256;
        if (TA) { kk = idx / BM; mm = idx % BM; }  // a[k*lda + m]: m contiguous
        else { mm = idx / BK; kk = idx % BK; }     // a[m*lda + k]: k contiguous
    };
    auto b_nk = [&](int i, int &nn, int &kk) {
        const int idx = t + i * 256;
        if (TB) { kk = idx / BN; nn = idx % BN; }  // b[k*ldb + n]
        else { nn = idx / BK; kk = idx % BK; }     // b[n*ldb + k] (Linear weight)
    };
    float ra[LPT], rb[LPT];
    auto load = [&](int64_t k0) {
#pragma unroll
        for (int i = 0; i < LPT; ++i) {
            int mm, kk, nn, kb;
            a_mk(i, mm, kk);
            b_nk(i, nn, kb);
            const int64_t gm = m0 + mm, gk = k0 + kk, gn = n0 + nn, gk2 = k0 + kb;
            ra[i] = (gm < M && gk < k_hi) ? (TA ? A[gk * lda + gm] : A[gm * lda + gk]) : 0.f;
            rb[i] = (gn < N && gk2 < k_hi) ? (TB ? B[gk2 * ldb + gn] : B[gn * ldb + gk2]) : 0.f;
        }
    };
    auto stage = [&](int buf) {
#pragma unroll
        for (int i = 0; i < LPT; ++i) {
            int mm, kk, nn, kb;
            a_mk(i, mm, kk);
            b_nk(i, nn, kb);
            As[buf][kk][mm] = ra[i];
            Bs[buf][kb][nn] = rb[i];
        }
    };
    int buf = 0;
    if (k_lo < k_hi) load(k_lo);
    for (int64_t k0 = k_lo; k0 < k_hi; k0 += BK) {
        stage(buf);
        __syncthreads();
        if (k0 + BK < k_hi) load(k0 + BK);  // next tile in flight under this tile's MFMAs
#pragma unroll
        for (int ks = 0; ks < BK; ks += 4) {
            const int kr = ks + (lane >> 4);
            float a[2], b[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) a[i] = As[buf][kr][wm * 32 + i * 16 + (lane & 15)];
#pragma unroll
            for (int j = 0; j < 2; ++j) b[j] = Bs[buf][kr][wn * 32 + j * 16 + (lane & 15)];
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
        }
        buf ^= 1;
    }
    // C/D map of 16x16x4: col = lane & 15, row = (lane >> 4) * 4 + reg
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int64_t gn = n0 + wn * 32 + j * 16 + (lane & 15);
            if (gn >= N) continue;
            const float bv = bias ? bias[gn] : 0.f;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t gm = m0 + wm * 32 + i * 16 + (lane >> 4) * 4 + r;
                if (gm < M) C[gm * ldc + gn] = acc[i][j][r] + bv;
            }
        }
}

// C[m, n] = bias[n] + sum_z W[z, m, n], z in order (deterministic split-K reduce)
__global__ void splitk_reduce(int64_t M, int64_t N, int S, const float *__restrict__ W,
                              const float *__restrict__ bias, float *__restrict__ C, int64_t ldc) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= M * N) return;
    const int64_t m = t / N, n = t - m * N;
    float s = 0.f;
    for (int z = 0; z < S; ++z) s += W[(int64_t)z * M * N + t];
    C[m * ldc + n] = s + (bias ? bias[n] : 0.f);
}

#ifndef IGR_GEMM_SPLIT_WG
#define IGR_GEMM_SPLIT_WG 512
#endif
#ifndef IGR_GEMM_SPLIT_MINK
#define IGR_GEMM_SPLIT_MINK 256
#endif
// Split count: enough workgroups to fill the chip when the output has few
// 64x64 tiles and K is long (e.g. a Linear weight gradient, K = node count).
static int split_count(int64_t m, int64_t n, int64_t k) {
    const int64_t tiles = ((m + BM - 1) / BM) * ((n + BN - 1) / BN);
    if (tiles >= 256 || k < 1024) return 1;
    int64_t s = (IGR_GEMM_SPLIT_WG + tiles - 1) / tiles;
    const int64_t smax = k / IGR_GEMM_SPLIT_MINK;  // at least this much of K per split
    if (s > smax) s = smax;
    if (s > 256) s = 256;
    return s < 1 ? 1 : (int)s;
}

}  // namespace igr

using namespace igr;

extern "C" int64_t igr_gemm_workspace_size(int64_t m, int64_t n, int64_t k) {
    const int s = (m > 0 && n > 0 && k > 0) ? split_count(m, n, k) : 1;
    return s > 1 ? (int64_t)s * m * n * (int64_t)sizeof(float) : 0;
}

extern "C" int igr_gemm_f32(int64_t m, int64_t n, int64_t k, const float *a, int64_t lda,
                            int32_t trans_a, const float *b, int64_t ldb, int32_t trans_b,
                            const float *bias, float *c, int64_t ldc, void *workspace, int64_t ws_bytes,
                            void *stream) {
    return guarded("igr_gemm_f32", [&]() -> int {
        const char *fn = "igr_gemm_f32";
        if (m < 0 || n < 0 || k < 0) return arg_error(fn, "negative size");
        if (ldc < n) return arg_error(fn, "ldc < n");
        if ((trans_a ? lda < m : lda < k) || (trans_b ? ldb < n : ldb < k))
            return arg_error(fn, "leading dimension too small");
        if (m == 0 || n == 0) return IGR_OK;
        if ((n + BN - 1) / BN > 65535) return arg_error(fn, "n too large");
        hipStream_t st = reinterpret_cast<hipStream_t>(stream);
        int S = split_count(m, n, k);
        if (S > 1 && (!workspace || ws_bytes < (int64_t)S * m * n * (int64_t)sizeof(float))) S = 1;
        const int64_t kc = S > 1 ? (((k + S - 1) / S + BK - 1) / BK) * BK : k;
        if (S > 1) S = (int)((k + kc - 1) / kc);  // BK-rounded slices may need fewer splits
        float *out = S > 1 ? static_cast<float *>(workspace) : c;
        const int64_t ldo = S > 1 ? n : ldc, zs = S > 1 ? m * n : 0;
        const float *bo = S > 1 ? nullptr : bias;
        dim3 grid((unsigned)((m + BM - 1) / BM), (unsigned)((n + BN - 1) / BN), (unsigned)S);
#define IGR_GEMM(TA_, TB_)                                                                                   \
    hipLaunchKernelGGL((gemm_f32_mfma<TA_, TB_>), grid, dim3(256), 0, st, m, n, k, a, lda, b, ldb, bo, out, ldo, \
                       kc, zs)
        if (trans_a && trans_b) IGR_GEMM(true, true);
        else if (trans_a) IGR_GEMM(true, false);
        else if (trans_b) IGR_GEMM(false, true);
        else IGR_GEMM(false, false);
#undef IGR_GEMM
        if (S > 1)
            hipLaunchKernelGGL(splitk_reduce, dim3((unsigned)((m * n + 255) / 256)), dim3(256), 0, st, m, n, S,
                               static_cast<const float *>(workspace), bias, c, ldc);
        return launch_status(fn);
    });
}
