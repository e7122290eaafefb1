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
#include <algorithm>
#include <type_traits>

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

// 128x128 output tile per workgroup for the large shapes (the Linear(d, 4d)
// projection over all nodes, the eval score GEMM): 4 waves of 64x64, each a 4x4
// grid of 16x16x4 MFMAs, so a K step reads 8 operands from LDS for 16 MFMAs.
// LDS images are laid out by the operand's global order so that staging stores
// and operand reads are both bank-conflict free: a k-contiguous operand (A not
// transposed, B a Linear weight) is kept [m][k] with stride BK+1, an
// m-contiguous one [k][m] with stride 128+16 (lanes 0-15 and 16-31 of an
// operand read sit 16 banks apart).  Double-buffered, next tile prefetched.
constexpr int BT = 128, BKT = 16, LPT2 = BT * BKT / 256;
constexpr int KSTR = BKT + 1, MSTR = BT + 16;

template <bool TRANS>  // TRANS: [k][x] image (x contiguous in global)
__device__ __forceinline__ int lds_idx(int x, int k) { return TRANS ? k * MSTR + x : x * KSTR + k; }

template <bool TA, bool TB>
__global__ __launch_bounds__(256) void gemm128_f32_mfma(int64_t M, int64_t N, int64_t K,
                                                        const float *__restrict__ A, int64_t lda,
                                                        const float *__restrict__ B, int64_t ldb,
                                                        const float *__restrict__ bias, float *__restrict__ C,
                                                        int64_t ldc) {
    constexpr int IMG = (BT * KSTR > BKT * MSTR) ? BT * KSTR : BKT * MSTR;
    // one allocation: the operand images, then (after the K loop) the C staging area over both
    __shared__ float smem[2 * 2 * IMG];
    float(*As)[IMG] = reinterpret_cast<float(*)[IMG]>(smem);
    float(*Bs)[IMG] = reinterpret_cast<float(*)[IMG]>(smem + 2 * IMG);
    const int t = threadIdx.x;
    const int lane = t & 63, wave = t >> 6;
    const int wm = wave >> 1, wn = wave & 1;  // 2x2 waves, 64x64 each
    const int64_t m0 = (int64_t)blockIdx.x * BT, n0 = (int64_t)blockIdx.y * BT;
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // staging coordinates: element i of this thread in a BT x BKT operand tile
    auto coord = [&](bool trans, int i, int &x, int &k) {
        const int idx = t + i * 256;
        if (trans) { k = idx / BT; x = idx % BT; }  // x contiguous in global
        else { x = idx / BKT; k = idx % BKT; }     // k contiguous in global
    };
    float ra[LPT2], rb[LPT2];
    auto load = [&](int64_t k0) {
#pragma unroll
        for (int i = 0; i < LPT2; ++i) {
            int x, k;
            coord(TA, i, x, k);
            const int64_t gm = m0 + x, gk = k0 + k;
            ra[i] = (gm < M && gk < K) ? (TA ? A[gk * lda + gm] : A[gm * lda + gk]) : 0.f;
            coord(TB, i, x, k);
            const int64_t gn = n0 + x, gk2 = k0 + k;
            rb[i] = (gn < N && gk2 < K) ? (TB ? B[gk2 * ldb + gn] : B[gn * ldb + gk2]) : 0.f;
        }
    };
    auto stage = [&](int buf) {
#pragma unroll
        for (int i = 0; i < LPT2; ++i) {
            int x, k;
            coord(TA, i, x, k);
            As[buf][lds_idx<TA>(x, k)] = ra[i];
            coord(TB, i, x, k);
            Bs[buf][lds_idx<TB>(x, k)] = rb[i];
        }
    };
    int buf = 0;
    if (K > 0) load(0);
    for (int64_t k0 = 0; k0 < K; k0 += BKT) {
        stage(buf);
        __syncthreads();
        if (k0 + BKT < K) load(k0 + BKT);
#pragma unroll
        for (int ks = 0; ks < BKT; ks += 4) {
            const int kr = ks + (lane >> 4);
            float a[4], b[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) a[i] = As[buf][lds_idx<TA>(wm * 64 + i * 16 + (lane & 15), kr)];
#pragma unroll
            for (int j = 0; j < 4; ++j) b[j] = Bs[buf][lds_idx<TB>(wn * 64 + j * 16 + (lane & 15), kr)];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
        }
        buf ^= 1;
    }
    // C through LDS: each wave stages 32 of its 64 rows at a time ([32][64+4]: the
    // two 16-lane halves of a store sit 16 banks apart), then writes whole 256-B
    // row segments with 16-B stores instead of 64-B pieces from 16 lanes.
    constexpr int CS = 68;
    float *Ws = smem + wave * 32 * CS;  // 4 x 8.5 KB within the 36 KB of operand images
    static_assert(4 * 32 * CS <= 2 * 2 * IMG, "C staging must fit in the operand images");
    const bool vec = (ldc % 4 == 0) && ((reinterpret_cast<uintptr_t>(C) & 15u) == 0);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        __syncthreads();  // every wave is past its last operand read (h = 0) / the previous half's reads
#pragma unroll
        for (int ii = 0; ii < 2; ++ii)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    Ws[(ii * 16 + (lane >> 4) * 4 + r) * CS + j * 16 + (lane & 15)] = acc[2 * h + ii][j][r];
        __syncthreads();
        const int c4 = (lane & 15) * 4;
        const int64_t gn = n0 + wn * 64 + c4;
        float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
        if (bias) {
            bv.x = gn < N ? bias[gn] : 0.f;
            bv.y = gn + 1 < N ? bias[gn + 1] : 0.f;
            bv.z = gn + 2 < N ? bias[gn + 2] : 0.f;
            bv.w = gn + 3 < N ? bias[gn + 3] : 0.f;
        }
#pragma unroll
        for (int pass = 0; pass < 8; ++pass) {
            const int row = pass * 4 + (lane >> 4);
            const int64_t gm = m0 + wm * 64 + h * 32 + row;
            if (gm >= M) continue;
            float4 v = *reinterpret_cast<const float4 *>(Ws + row * CS + c4);
            v = make_float4(v.x + bv.x, v.y + bv.y, v.z + bv.z, v.w + bv.w);
            float *cp = C + gm * ldc + gn;
            if (vec && gn + 3 < N) {
                *reinterpret_cast<float4 *>(cp) = v;
            } else {
                if (gn < N) cp[0] = v.x;
                if (gn + 1 < N) cp[1] = v.y;
                if (gn + 2 < N) cp[2] = v.z;
                if (gn + 3 < N) cp[3] = v.w;
            }
        }
    }
}

// Tall-and-skinny projection with the WEIGHT HELD IN REGISTERS:
//   C[M, N] = A[M, K] W^T + bias,  K in {32, 64}, N a multiple of 64, M = node count
// (AttIGCN's Linear(d, 4d) over every node, model.py:4259, 4264; NGCF's Linear(d, d),
// model.py:4039).  With K this short a conventional tile has only K / 16 steps to
// hide its first loads and its C epilogue behind; here a workgroup is persistent
// over 64-row tiles of A instead:
//  * each wave owns 16 NB output columns and keeps its slice of W as MFMA
//    operands in K/4 * NB registers for the whole launch (W never touches LDS);
//  * the MFMA is issued transposed, D = W_slice (16 x 4) x A_tile^T (4 x 16), so a
//    lane ends up with FOUR CONSECUTIVE COLUMNS of one output row: C leaves the
//    registers as 16-byte stores with no LDS staging;
//  * A tiles go global -> registers -> LDS (double-buffered, the tile after next
//    loaded while the next one is computed, one barrier per tile), stride K + 4
//    floats so both the 16-byte staging stores and the operand reads are
//    bank-conflict free;
//  * a tile is computed as two halves of 32 rows with accumulator sets of their own,
//    and the C stores of one half are spread through the MFMAs of the NEXT half (one
//    16-byte store instruction per two k steps) instead of a burst of 2 NB stores
//    after each half: a wave issues in order, so a burst holds its MFMAs back for as
//    long as the store queue takes to accept it, on all four SIMDs at once;
//  * the only wait on memory is the one before the next tile goes to LDS; memory
//    operations retire in order and those loads are older than the stores that
//    follow them, so C drains under the MFMAs;
//  * bias is the accumulators' initial value.
// Rows past M are never stored; loads clamp the row index, so every tile is read
// with straight-line code.  Two workgroups per CU.
// A tile of TM rows x K floats: global -> registers (row index clamped to M - 1, so the
// code is straight-line for every tile) and registers -> LDS image with row stride K + 4.
template <int K, int LP>
__device__ __forceinline__ void rows_tile_load(f32x4 (&ra)[LP], const float *__restrict__ A, int64_t lda, int64_t M,
                                               int64_t m0, int t) {
#pragma unroll
    for (int i = 0; i < LP; ++i) {
        const int idx = t + i * 256;
        int64_t gm = m0 + idx / (K / 4);
        gm = gm < M ? gm : M - 1;
        ra[i] = *reinterpret_cast<const f32x4 *>(A + gm * lda + (idx % (K / 4)) * 4);
    }
}
template <int K, int LP>
__device__ __forceinline__ void rows_tile_stage(const f32x4 (&ra)[LP], float *as, int t) {
#pragma unroll
    for (int i = 0; i < LP; ++i) {
        const int idx = t + i * 256;
        *reinterpret_cast<f32x4 *>(as + (idx / (K / 4)) * (K + 4) + (idx % (K / 4)) * 4) = ra[i];
    }
}

#ifndef IGR_GEMMP_OCC
#define IGR_GEMMP_OCC 2
#endif
#ifndef IGR_GEMMP_PIN
#define IGR_GEMMP_PIN 0x106
#endif
template <int KS, int NB, bool TB>
__global__ __launch_bounds__(256, IGR_GEMMP_OCC) void gemm_rows_persistent(int64_t M, const float *__restrict__ A,
                                                                         int64_t lda, const float *__restrict__ B,
                                                                         int64_t ldb, const float *__restrict__ bias,
                                                                         float *__restrict__ C, int64_t ldc) {
    constexpr int K = KS * 4, TM = 64, STR = K + 4;
    constexpr int LP = TM * K / 4 / 256;
    constexpr int NST = 2 * NB;          // store instructions per half
    constexpr int GAP = KS / NST > 0 ? KS / NST : 1;  // k steps between two of them
    __shared__ __align__(16) float As[2][TM * STR];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int m16 = lane & 15, g = lane >> 4;
    const int64_t n0 = (int64_t)blockIdx.y * (64 * NB) + wave * (16 * NB);
    const int64_t n_tiles = (M + TM - 1) / TM, full_tiles = M / TM;
    int64_t tile = blockIdx.x;
    if (tile >= n_tiles) return;  // the whole workgroup leaves together, before any barrier
    float w[NB][KS];
    f32x4 bz[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
        const int64_t n = n0 + 16 * j + m16;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const int k = 4 * ks + g;
            w[j][ks] = TB ? B[(int64_t)k * ldb + n] : B[n * ldb + k];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) bz[j][r] = bias ? bias[n0 + 16 * j + 4 * g + r] : 0.f;
    }
    f32x4 ra[LP];  // a native vector: a struct float4 would be copied with memcpy and stay in scratch
    auto load = [&](int64_t m0) __attribute__((always_inline)) { rows_tile_load<K, LP>(ra, A, lda, M, m0, t); };
    auto stage = [&](int b) __attribute__((always_inline)) { rows_tile_stage<K, LP>(ra, As[b], t); };
    // one store instruction: columns 16 j + 4 g .. + 3 of row m0 + 16 rb + m16
    auto store1 = [&](const f32x4 (&src)[NB][2], int64_t m0, int s, auto guard) __attribute__((always_inline)) {
        const int rb = s / NB, j = s % NB;
        const int64_t gm = m0 + 16 * rb + m16;
        if (!decltype(guard)::value || gm < M)
            *reinterpret_cast<f32x4 *>(C + gm * ldc + n0 + 16 * j + 4 * g) = src[j][rb];
    };
    // MFMAs of rows [32 half, 32 half + 32) of the tile in As[buf] into dst; when STORE, the
    // 2 NB stores of `src` (rows m0 ...) are issued one every GAP k steps on the way
    auto half_pass = [&](int buf, int half, f32x4 (&dst)[NB][2], const f32x4 (&src)[NB][2], int64_t m0,
                         auto do_store, auto guard) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < NB; ++j)
#pragma unroll
            for (int rb = 0; rb < 2; ++rb) dst[j][rb] = bz[j];
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
            for (int rb = 0; rb < 2; ++rb) {
                const float a = As[buf][(16 * (2 * half + rb) + m16) * STR + 4 * ks + g];
#pragma unroll
                for (int j = 0; j < NB; ++j)
                    dst[j][rb] = __builtin_amdgcn_mfma_f32_16x16x4f32(w[j][ks], a, dst[j][rb], 0, 0, 0);
            }
            if (decltype(do_store)::value && ks % GAP == GAP - 1 && ks / GAP < NST) {
                store1(src, m0, ks / GAP, guard);
                // keep the store where it stands: without this the scheduler gathers the
                // stores of a half back into one burst.  LDS reads, VALU and SALU may cross.
                __builtin_amdgcn_sched_barrier(IGR_GEMMP_PIN);
            }
        }
        if (decltype(do_store)::value)
#pragma unroll
            for (int s = KS / GAP; s < NST; ++s) store1(src, m0, s, guard);
    };
    f32x4 acc0[NB][2], acc1[NB][2];
    load(tile * TM);
    stage(0);
    // the weight slice, the bias and the first tile are complete here: no wait inside
    // the loop ever has to count them
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    load((tile + gridDim.x) * TM);
    half_pass(0, 0, acc0, acc1, 0, std::false_type{}, std::false_type{});
    int buf = 0;
    auto step = [&](auto guard) __attribute__((always_inline)) {
        // half 1 of this tile while half 0 leaves
        half_pass(buf, 1, acc1, acc0, tile * TM, std::true_type{}, guard);
        stage(buf ^ 1);  // the next tile; every wave left that buffer before the last barrier
        __syncthreads();
        load((tile + 2 * gridDim.x) * TM);
        // half 0 of the next tile while half 1 of this one leaves
        half_pass(buf ^ 1, 0, acc0, acc1, tile * TM + 32, std::true_type{}, guard);
        buf ^= 1;
    };
    for (; tile + gridDim.x < full_tiles; tile += gridDim.x) step(std::false_type{});
    for (; tile + gridDim.x < n_tiles; tile += gridDim.x) step(std::true_type{});
    // the last tile of this workgroup
    half_pass(buf, 1, acc1, acc0, tile * TM, std::true_type{}, std::true_type{});
#pragma unroll
    for (int s = 0; s < NST; ++s) store1(acc1, tile * TM + 32, s, std::true_type{});
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
#ifndef IGR_GEMM128
#define IGR_GEMM128 1
#endif
        // the register-resident-weight kernel: short K, N in whole 64-column groups
        const bool rows_ok = !trans_a && S == 1 && (k == 32 || k == 64 || k == 128) && n % 64 == 0 && m >= 1024 &&
                             lda % 4 == 0 && ldc % 4 == 0 && aligned16(a) && aligned16(c) && n / 64 <= 65535;
        if (rows_ok) {
            const int64_t tiles = (m + 63) / 64;
            // wider column groups per workgroup once there are enough row tiles to fill the chip
            int nb = (n % 256 == 0 && tiles >= 512) ? 4 : ((n % 128 == 0 && tiles * 2 >= 512) ? 2 : 1);
            if (k == 128 && nb > 2) nb = 2;  // twice the weight registers per column group
            static int cus = 0;
            if (cus <= 0) {
                int dev = 0;
                if (hipGetDevice(&dev) != hipSuccess ||
                    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
                    cus = 256;
            }
            const int64_t gy = n / (64 * nb);
            const int64_t gx = std::min<int64_t>(tiles, std::max<int64_t>(1, IGR_GEMMP_OCC * (int64_t)cus / gy));
            dim3 gp((unsigned)gx, (unsigned)gy);
#define IGR_GEMMP(KS_, NB_)                                                                                       \
    do {                                                                                                          \
        if (trans_b)                                                                                              \
            hipLaunchKernelGGL((gemm_rows_persistent<KS_, NB_, true>), gp, dim3(256), 0, st, m, a, lda, b, ldb,   \
                               bias, c, ldc);                                                                     \
        else                                                                                                      \
            hipLaunchKernelGGL((gemm_rows_persistent<KS_, NB_, false>), gp, dim3(256), 0, st, m, a, lda, b, ldb,  \
                               bias, c, ldc);                                                                     \
    } while (0)
            if (k == 128) {
                if (nb == 2) IGR_GEMMP(32, 2); else IGR_GEMMP(32, 1);
            } else if (k == 64) {
                if (nb == 4) IGR_GEMMP(16, 4); else if (nb == 2) IGR_GEMMP(16, 2); else IGR_GEMMP(16, 1);
            } else {
                if (nb == 4) IGR_GEMMP(8, 4); else if (nb == 2) IGR_GEMMP(8, 2); else IGR_GEMMP(8, 1);
            }
#undef IGR_GEMMP
            return launch_status(fn);
        }
        // 128 tiles only when they still give >= 2048 workgroups (8 per CU): on
        // small shapes the 64 tiles' extra parallelism wins (measured)
        const int64_t tiles128 = ((m + BT - 1) / BT) * ((n + BT - 1) / BT);
        if (IGR_GEMM128 && S == 1 && tiles128 >= 2048 && (n + BT - 1) / BT <= 65535) {
            dim3 g2((unsigned)((m + BT - 1) / BT), (unsigned)((n + BT - 1) / BT));
#define IGR_GEMM2(TA_, TB_) \
    hipLaunchKernelGGL((gemm128_f32_mfma<TA_, TB_>), g2, dim3(256), 0, st, m, n, k, a, lda, b, ldb, bias, c, ldc)
            if (trans_a && trans_b) IGR_GEMM2(true, true);
            else if (trans_a) IGR_GEMM2(true, false);
            else if (trans_b) IGR_GEMM2(false, true);
            else IGR_GEMM2(false, false);
#undef IGR_GEMM2
            return launch_status(fn);
        }
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
