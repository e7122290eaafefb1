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
// Both: a wave per destination row - or, following the graph's row schedule, per chunk of
// a split row and per unsplit row, heaviest first (a hub row is otherwise one wave's
// loop) - d / 4 lanes per source row (one 16-byte load per lane), 64 / (d / 4) edges side
// by side, several edges per lane group in flight.
#include "common.h"

namespace igr {

// Edges per lane group per trip (0: chosen per width so that a trip covers 16 edges,
// at most 4 per group) and trips whose gathers are all issued before the first of them
// is reduced (a scheduling barrier keeps them there).  A trip's loads are
// unconditional - an empty slot re-reads the row's last edge, an L2 hit - because a
// load under a lane condition whose other arm zeroes the register is followed by a
// wait at the join: with such loads the kernel ran with one 16-byte gather in flight
// per lane (24.5 ms at nnz 411 M, h = 4, d = 64, and slower the more edges a trip took).
// Measured on MI355X with the loads unconditional (U x NT): 1x4 19.8 ms, 4x1 19.8, 2x2 19.9,
// 2x3 20.0, 1x6 20.2, 4x2 20.3, 1x8 20.4, 1x2 21.2, 4x4 23.5 (133 VGPRs: 3 waves per SIMD).
#ifndef IGR_SDDMM_SHARED_U
#define IGR_SDDMM_SHARED_U 1
#endif
#ifndef IGR_SDDMM_SHARED_NT
#define IGR_SDDMM_SHARED_NT 4
#endif
static_assert(IGR_SDDMM_SHARED_NT >= 1 && IGR_SDDMM_SHARED_NT <= 8, "1 to 8 trips per pass");

typedef float v4f __attribute__((ext_vector_type(4)));

// x of the lane that a DPP control selects (quad permutes and row mirrors: every
// lane has a source, no LDS traffic)
template <int CTRL>
__device__ __forceinline__ float dpp_f(float x) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xf, 0xf, true));
}

// Sum of x over the LPE (a power of two) consecutive lanes of a group, left in every one
// of them: xor 1 and xor 2 inside quads, then the mirrored half of 8 and of 16 lanes
// (the partial sums are uniform inside what is mirrored), shuffles beyond a row.
template <int LPE>
__device__ __forceinline__ float group_sum(float x) {
    if (LPE >= 2) x += dpp_f<0xB1>(x);   // quad_perm [1, 0, 3, 2]
    if (LPE >= 4) x += dpp_f<0x4E>(x);   // quad_perm [2, 3, 0, 1]
    if (LPE >= 8) x += dpp_f<0x141>(x);  // row_half_mirror
    if (LPE >= 16) x += dpp_f<0x140>(x); // row_mirror
    if (LPE >= 32) x += shfl_xor_f(x, 16);
    if (LPE >= 64) x += shfl_xor_f(x, 32);
    return x;
}

// Four per-lane partial sums (one per head) over the LPE lanes of a group, reduced so that
// each lane ends with the FULL sum of ONE head instead of every lane with all four: a
// butterfly - lanes of a pair exchange the two heads the other one keeps (xor 1), then the
// one (xor 2), then the single value is added across the quads (mirrored halves, shuffles
// beyond a 16-lane row).  Lane `sub` of the group ends with head head4_of(sub).  Odd quads
// hold the heads in reverse order, so that a lane's partner under a row mirror (i <-> 7 - i,
// i <-> 15 - i) holds the same head.  11 lane operations instead of 16, and the result is
// laid out for one coalesced 4-byte store per lane.
__device__ __forceinline__ int head4_of(int sub) { return (sub & 3) ^ ((sub & 4) ? 3 : 0); }

template <int LPE>
__device__ __forceinline__ float group_sum_heads4(float s0, float s1, float s2, float s3, bool b0, bool b1) {
    static_assert(LPE >= 8, "a group spans at least two quads");
    const float k01 = (b0 ? s1 : s0) + dpp_f<0xB1>(b0 ? s0 : s1);  // head b0
    const float k23 = (b0 ? s3 : s2) + dpp_f<0xB1>(b0 ? s2 : s3);  // head 2 + b0
    float x = (b1 ? k23 : k01) + dpp_f<0x4E>(b1 ? k01 : k23);     // head 2 b1 + b0, over the quad
    x += dpp_f<0x141>(x);                 // row_half_mirror: the other quad of the 8
    if (LPE >= 16) x += dpp_f<0x140>(x);  // row_mirror: the other 8 of the 16
    if (LPE >= 32) x += shfl_xor_f(x, 16);
    if (LPE >= 64) x += shfl_xor_f(x, 32);
    return x;
}

template <int D, int H, bool EID>
struct SddmmShared {
    static constexpr int LPE = D / 4;    // lanes per edge (source row)
    static constexpr int EPW = 64 / LPE; // edges side by side in a wave
    static constexpr int UE = IGR_SDDMM_SHARED_U > 0 ? IGR_SDDMM_SHARED_U : (16 / EPW < 1 ? 1 : (16 / EPW > 4 ? 4 : 16 / EPW));
    static constexpr int TRIP = UE * EPW;  // edges per trip (divides 64)
    static constexpr int NT = IGR_SDDMM_SHARED_NT < 64 / TRIP ? IGR_SDDMM_SHARED_NT : 64 / TRIP;  // trips per pass

    // H = 4, one edge per group and trip: the butterfly leaves lane `sub` of group eg with one
    // head of the trip's edge; the lanes whose quad index (sub >> 2) equals the trip's index
    // inside a run of QT = LPE / 4 trips keep it, so after QT trips the 64 lanes hold the
    // QT * EPW * 4 = 64 scores of QT * EPW consecutive edges - one 256-byte run of `out`,
    // written by ONE store with every lane active instead of four 16-byte stores from one
    // lane in sixteen (19.8 -> 19.1 ms at nnz 411 M, h = 4, d = 64; the launch takes 16.0 ms
    // with no stores at all, so most of what the 6.6 GB of scores cost is not their shape).
    template <int NTR>
    static __device__ __forceinline__ void pass_heads4(int t0, int n, int cl, int eg, int sub, const v4f (&uq)[H],
                                                       const float *__restrict__ vs, int ld_v,
                                                       const int64_t *__restrict__ eid, int64_t base,
                                                       float *__restrict__ out) {
        constexpr int QT = LPE / 4;                    // trips per store
        constexpr int NS = (NTR + QT - 1) / QT;        // stores of this pass
        const int hd = head4_of(sub);  // the head this lane ends up holding
        const bool b0 = (hd & 1) != 0, b1 = (hd & 2) != 0;
        const int quad = sub >> 2;
        v4f vk[NTR];
#pragma unroll
        for (int tt = 0; tt < NTR; ++tt) {
            const int k = t0 + tt * EPW + eg;
            const int c = shfl_i(cl, k < n ? k : n - 1);
            vk[tt] = *reinterpret_cast<const v4f *>(vs + (int64_t)c * ld_v);
        }
        __builtin_amdgcn_sched_barrier(0);
        float keep[NS];
#pragma unroll
        for (int q = 0; q < NS; ++q) keep[q] = 0.f;
#pragma unroll
        for (int tt = 0; tt < NTR; ++tt) {
            float s[4];
#pragma unroll
            for (int hh = 0; hh < 4; ++hh)
                s[hh] = uq[hh].x * vk[tt].x + uq[hh].y * vk[tt].y + uq[hh].z * vk[tt].z + uq[hh].w * vk[tt].w;
            const float x = group_sum_heads4<LPE>(s[0], s[1], s[2], s[3], b0, b1);
            if (quad == tt % QT) keep[tt / QT] = x;
        }
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            const int k = t0 + (q * QT + quad) * EPW + eg;  // the edge whose score this lane kept
            // q QT + quad < NTR: the lane kept a trip of THIS pass (a wide group has more quads than trips)
            if (q * QT + quad < NTR && k < n) {
                out[(EID ? eid[base + k] : base + k) * 4 + hd] = keep[q];
            }
        }
    }

    // NTR trips starting at edge t0 of the block: every gather first, then each trip's
    // dots, their sums over the group's lanes and the stores (lane 0 of the group
    // writes the H scores of each of its UE edges)
    template <int NTR>
    static __device__ __forceinline__ void pass(int t0, int n, int cl, int eg, int sub, const v4f (&uq)[H],
                                                const float *__restrict__ vs, int ld_v,
                                                const int64_t *__restrict__ eid, int64_t base,
                                                float *__restrict__ out) {
        if constexpr (H == 4 && UE == 1 && LPE >= 8) {
            pass_heads4<NTR>(t0, n, cl, eg, sub, uq, vs, ld_v, eid, base, out);
            return;
        }
        v4f vk[NTR][UE];
#pragma unroll
        for (int tt = 0; tt < NTR; ++tt)
#pragma unroll
            for (int j = 0; j < UE; ++j) {
                const int k = t0 + tt * TRIP + eg * UE + j;
                const int c = shfl_i(cl, k < n ? k : n - 1);
                vk[tt][j] = *reinterpret_cast<const v4f *>(vs + (int64_t)c * ld_v);
            }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int tt = 0; tt < NTR; ++tt) {
            const int k0 = t0 + tt * TRIP + eg * UE;
            float sv[UE][H];
#pragma unroll
            for (int j = 0; j < UE; ++j)
#pragma unroll
                for (int hh = 0; hh < H; ++hh)
                    sv[j][hh] = group_sum<LPE>(uq[hh].x * vk[tt][j].x + uq[hh].y * vk[tt][j].y +
                                               uq[hh].z * vk[tt][j].z + uq[hh].w * vk[tt][j].w);
            if (sub == 0) {
#pragma unroll
                for (int j = 0; j < UE; ++j) {
                    const int k = k0 + j;
                    if (k >= n) continue;
                    float *o = out + (EID ? eid[base + k] : base + k) * H;
                    if (H % 4 == 0) {
#pragma unroll
                        for (int q = 0; q < H / 4; ++q)
                            reinterpret_cast<v4f *>(o)[q] = v4f{sv[j][4 * q], sv[j][4 * q + 1], sv[j][4 * q + 2], sv[j][4 * q + 3]};
                    } else {
#pragma unroll
                        for (int hh = 0; hh < H; ++hh) o[hh] = sv[j][hh];
                    }
                }
            }
        }
    }
};

constexpr int kXcds = 8;
constexpr int kXcdStrip = 32;  // workgroups (128 rows) per strip

template <int D, int H, bool EID, bool PLAN>
__global__ __launch_bounds__(256) void sddmm_shared_kernel(int64_t n_rows, const int64_t *__restrict__ row_ptr,
                                                           const int32_t *__restrict__ col,
                                                           const int64_t *__restrict__ eid, RowPlan plan,
                                                           const float *__restrict__ u, int64_t ld_u,
                                                           const float *__restrict__ v, int ld_v,
                                                           float *__restrict__ out) {
    using S = SddmmShared<D, H, EID>;
    int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (!PLAN) {
        // natural row order: workgroups are dealt to the 8 XCDs round-robin, so they are
        // renumbered for each XCD to walk strips of kXcdStrip consecutive workgroups' rows
        // (the grid is a whole number of 8-strip groups).  The scores of neighbouring rows
        // share 128-byte lines, and a line written half through one XCD's L2 and half
        // through another's reaches memory twice.  Strips, not one range per XCD: the
        // heavy rows of a bipartite graph sit together (the item rows: half of the edges in
        // a tenth of the rows), and the XCD that owned them all would finish 2.6 times later.
        const int64_t q = blockIdx.x / kXcds;
        const int64_t lb = (q / kXcdStrip) * (kXcds * kXcdStrip) + (int64_t)(blockIdx.x % kXcds) * kXcdStrip +
                           q % kXcdStrip;
        w = lb * 4 + (threadIdx.x >> 6);
    }
    int64_t r, b, e;
    if (PLAN) {
        if (w >= plan.n_chunks + plan.n_order) return;
        if (w < plan.n_chunks) {
            r = plan.chunk_row[w];
            b = plan.chunk_beg[w];
            e = min(b + plan.chunk_edges, row_ptr[r + 1]);
        } else {
            r = plan.order[w - plan.n_chunks];
            b = row_ptr[r];
            e = row_ptr[r + 1];
        }
    } else {
        r = w;
        if (r >= n_rows) return;
        b = row_ptr[r];
        e = row_ptr[r + 1];
    }
    const int lane = threadIdx.x & 63;
    const int eg = lane / S::LPE;
    const int sub = lane - eg * S::LPE;
    v4f uq[H];
#pragma unroll
    for (int hh = 0; hh < H; ++hh) uq[hh] = *reinterpret_cast<const v4f *>(u + r * ld_u + hh * D + sub * 4);
    const float *vs = v + sub * 4;
    for (int64_t base = b; base < e; base += 64) {
        const int n = (int)min((int64_t)64, e - base);
        const int cl = lane < n ? col[base + lane] : 0;
        // n is the same in every lane: the number of trips left picks a straight-line pass
        for (int t0 = 0; t0 < n; t0 += S::NT * S::TRIP) {
            const int left = (n - t0 + S::TRIP - 1) / S::TRIP;
            const int nt = left < S::NT ? left : S::NT;
#define IGR_PASS(N_) S::template pass<(S::NT >= N_ ? N_ : 1)>(t0, n, cl, eg, sub, uq, vs, ld_v, eid, base, out)
            if (nt == 8) IGR_PASS(8);
            else if (nt == 7) IGR_PASS(7);
            else if (nt == 6) IGR_PASS(6);
            else if (nt == 5) IGR_PASS(5);
            else if (nt == 4) IGR_PASS(4);
            else if (nt == 3) IGR_PASS(3);
            else if (nt == 2) IGR_PASS(2);
            else IGR_PASS(1);
#undef IGR_PASS
        }
    }
}

// Edges per lane group per trip of the gradient kernel, measured on MI355X (nnz 411 M,
// h = 4, d = 64): 1 -> 19.4 ms, 2 -> 18.6, 4 -> 19.6, 8 -> 22.8.
#ifndef IGR_SPMM_SHARED_U
#define IGR_SPMM_SHARED_U 2
#endif
// y[r, hh, :] = sum over the edges of row r of rhs[eid, hh] * x[col, :]: each source row
// is gathered once and feeds H accumulators; the EPW lane groups take alternate edges
// and are summed in a fixed xor tree at the end (deterministic).
// With a row plan (PLAN) a wave takes one chunk of a split row, whose partial sums go to
// its slot of `ws` (H * D floats per chunk; heads_combine_kernel adds a row's slots in
// chunk order), or one whole unsplit row, heaviest first.
template <int D, int H, bool PLAN>
__global__ __launch_bounds__(256) void spmm_shared_heads_kernel(int64_t n_rows, const int64_t *__restrict__ row_ptr,
                                                                const int32_t *__restrict__ col,
                                                                const int64_t *__restrict__ eid, RowPlan plan,
                                                                const float *__restrict__ x, int ldx,
                                                                const float *__restrict__ rhs,
                                                                float *__restrict__ y, int64_t ldy,
                                                                float *__restrict__ ws) {
    constexpr int LPE = D / 4;
    constexpr int EPW = 64 / LPE;
    constexpr int UE = IGR_SPMM_SHARED_U;
    constexpr int TRIP = UE * EPW;
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    int64_t b, e;
    float *dst;
    if (PLAN) {
        if (w >= plan.n_chunks + plan.n_order) return;
        if (w < plan.n_chunks) {
            const int64_t r = plan.chunk_row[w];
            b = plan.chunk_beg[w];
            e = min(b + plan.chunk_edges, row_ptr[r + 1]);
            dst = ws + w * (int64_t)(H * D);
        } else {
            const int64_t r = plan.order[w - plan.n_chunks];
            b = row_ptr[r];
            e = row_ptr[r + 1];
            dst = y + r * ldy;
        }
    } else {
        if (w >= n_rows) return;
        b = row_ptr[w];
        e = row_ptr[w + 1];
        dst = y + w * ldy;
    }
    const int lane = threadIdx.x & 63;
    const int eg = lane / LPE;
    const int sub = lane - eg * LPE;
    const float *xs = x + sub * 4;
    float4 acc[H];
#pragma unroll
    for (int hh = 0; hh < H; ++hh) acc[hh] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t base = b; base < e; base += 64) {
        const int n = (int)min((int64_t)64, e - base);
        const int cl = lane < n ? col[base + lane] : 0;
        const int64_t el = lane < n ? (eid ? eid[base + lane] : base + lane) : 0;
        for (int t = 0; t < n; t += TRIP) {
            const int k0 = t + eg * UE;
            v4f xv[UE];
            v4f wq[UE][(H + 3) / 4];
            float wv[UE][H];
            // every load of the trip is unconditional (an empty slot re-reads the row's last
            // edge and its weights are replaced by zeros), so all of them are in flight at once
#pragma unroll
            for (int j = 0; j < UE; ++j) {
                const int src = k0 + j < n ? k0 + j : n - 1;
                const int c = shfl_i(cl, src);
                const int64_t ee = ((int64_t)shfl_i((int)(el >> 32), src) << 32) | (uint32_t)shfl_i((int)el, src);
                xv[j] = *reinterpret_cast<const v4f *>(xs + (int64_t)c * ldx);
                if (H % 4 == 0) {
#pragma unroll
                    for (int q = 0; q < H / 4; ++q) wq[j][q] = reinterpret_cast<const v4f *>(rhs + ee * H)[q];
                } else {
#pragma unroll
                    for (int hh = 0; hh < H; ++hh) wv[j][hh] = rhs[ee * H + hh];
                }
            }
#pragma unroll
            for (int j = 0; j < UE; ++j) {
                const bool valid = k0 + j < n;
#pragma unroll
                for (int hh = 0; hh < H; ++hh) {
                    const float w = H % 4 == 0 ? wq[j][hh / 4][hh % 4] : wv[j][hh];
                    const float wz = valid ? w : 0.f;
                    acc[hh].x = fmaf(wz, xv[j].x, acc[hh].x);
                    acc[hh].y = fmaf(wz, xv[j].y, acc[hh].y);
                    acc[hh].z = fmaf(wz, xv[j].z, acc[hh].z);
                    acc[hh].w = fmaf(wz, xv[j].w, acc[hh].w);
                }
            }
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
        for (int hh = 0; hh < H; ++hh) *reinterpret_cast<float4 *>(dst + hh * D + sub * 4) = acc[hh];
    }
}

// y[split_row[s], :] = the sum of the row's chunk partials (one block per split row;
// width = H * D floats <= 512, one float4 column group per thread).  The block's
// 256 / (width / 4) slots take alternate chunks - a hub row has thousands - and are
// added in slot order through LDS: a fixed order, the same bits on every run.
__global__ __launch_bounds__(256) void heads_combine_kernel(int64_t n_split, const int32_t *__restrict__ split_row,
                                                            const int64_t *__restrict__ split_ptr,
                                                            const float *__restrict__ ws, int width,
                                                            float *__restrict__ y, int64_t ldy) {
    __shared__ float4 red[256];
    const int64_t s = blockIdx.x;
    const int cols = width / 4;          // 8 ... 128, a power of two
    const int slots = 256 / cols;
    const int slot = threadIdx.x / cols;
    const int t = threadIdx.x - slot * cols;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (s < n_split) {
        for (int64_t k = split_ptr[s] + slot; k < split_ptr[s + 1]; k += slots) {
            const float4 p = *reinterpret_cast<const float4 *>(ws + k * width + t * 4);
            acc.x += p.x;
            acc.y += p.y;
            acc.z += p.z;
            acc.w += p.w;
        }
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    if (s >= n_split || slot != 0) return;
    for (int k = 1; k < slots; ++k) {
        const float4 p = red[k * cols + t];
        acc.x += p.x;
        acc.y += p.y;
        acc.z += p.z;
        acc.w += p.w;
    }
    *reinterpret_cast<float4 *>(y + (int64_t)split_row[s] * ldy + t * 4) = acc;
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
        const RowPlan plan = row_plan_of(g);
        const bool planned = use_row_plan(g);
        const int64_t waves = planned ? g->n_chunks + g->n_order : g->n_rows;
        int64_t blocks = (waves + 3) / 4;
        if (!planned) {  // whole groups of 8 strips: every renumbered workgroup below the count is taken
            const int64_t group = (int64_t)kXcds * kXcdStrip;
            blocks = (blocks + group - 1) / group * group;
        }
        const dim3 grid((unsigned)blocks);
#define IGR_GO(EID_, PLAN_)                                                                                    \
    hipLaunchKernelGGL((sddmm_shared_kernel<D, H, EID_, PLAN_>), grid, dim3(256), 0, st, g->n_rows, g->row_ptr, \
                       g->col_idx, g->edge_id, plan, u, ld_u, v, (int)ld_v, out)
        if (g->edge_id) {
            if (planned) IGR_GO(true, true);
            else IGR_GO(true, false);
        } else {
            if (planned) IGR_GO(false, true);
            else IGR_GO(false, false);
        }
#undef IGR_GO
    }
};

template <int D, int H>
struct LaunchSpmmShared {
    static void go(const igr_csr *g, const float *x, int64_t ldx, const float *rhs, float *y, int64_t ldy,
                   float *ws, hipStream_t st) {
        const RowPlan plan = row_plan_of(g);
        // split rows need the workspace for their chunk partials; without one every row is one wave's
        const bool planned = use_row_plan(g) && (g->n_chunks == 0 || ws != nullptr);
        const int64_t waves = planned ? g->n_chunks + g->n_order : g->n_rows;
        const dim3 grid((unsigned)((waves + 3) / 4));
        if (planned) {
            hipLaunchKernelGGL((spmm_shared_heads_kernel<D, H, true>), grid, dim3(256), 0, st, g->n_rows, g->row_ptr,
                               g->col_idx, g->edge_id, plan, x, (int)ldx, rhs, y, ldy, ws);
            if (g->n_split > 0)
                hipLaunchKernelGGL(heads_combine_kernel, dim3((unsigned)g->n_split), dim3(256), 0, st, g->n_split,
                                   g->split_row, g->split_ptr, ws, H * D, y, ldy);
        } else {
            hipLaunchKernelGGL((spmm_shared_heads_kernel<D, H, false>), grid, dim3(256), 0, st, g->n_rows, g->row_ptr,
                               g->col_idx, g->edge_id, plan, x, (int)ldx, rhs, y, ldy, ws);
        }
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
        if (ld_v > 2147483647) return arg_error(fn, "ld_v too large");
        if (h % 4 == 0 && !aligned16(out)) return arg_error(fn, "out must be 16-byte aligned");
        if (!dispatch_dh<LaunchSddmmShared>(d, h, g, u, ld_u, v, ld_v, out, reinterpret_cast<hipStream_t>(stream)))
            return arg_error(fn, "supported: d in {32, 64, 128, 256} with h * d <= 512, h a power of two");
        return launch_status(fn);
    });
}

extern "C" int igr_spmm_shared_heads_f32(const igr_csr *g, int32_t h, int32_t d, const float *x, int64_t ldx,
                                         const float *rhs, float *y, int64_t ldy, void *stream) {
    return igr_spmm_shared_heads_ws_f32(g, h, d, x, ldx, rhs, y, ldy, nullptr, 0, stream);
}

extern "C" int64_t igr_spmm_shared_heads_workspace_size(const igr_csr *g, int32_t h, int32_t d) {
    if (!g || h <= 0 || d <= 0 || g->n_chunks <= 0) return 0;
    return g->n_chunks * (int64_t)h * d * (int64_t)sizeof(float);
}

extern "C" int igr_spmm_shared_heads_ws_f32(const igr_csr *g, int32_t h, int32_t d, const float *x, int64_t ldx,
                                            const float *rhs, float *y, int64_t ldy, float *workspace,
                                            int64_t workspace_bytes, void *stream) {
    return guarded("igr_spmm_shared_heads_ws_f32", [&]() -> int {
        const char *fn = "igr_spmm_shared_heads_ws_f32";
        if (workspace && g && workspace_bytes < igr_spmm_shared_heads_workspace_size(g, h, d))
            return arg_error(fn, "workspace smaller than igr_spmm_shared_heads_workspace_size");
        if (workspace && !aligned16(workspace)) return arg_error(fn, "workspace must be 16-byte aligned");
        if (!g || h <= 0 || d <= 0) return arg_error(fn, "bad graph / h / d");
        if (ldx < d || ldy < (int64_t)h * d) return arg_error(fn, "leading dimension too small");
        if (g->n_rows == 0) return IGR_OK;
        if (!y || (g->nnz > 0 && (!x || !rhs))) return arg_error(fn, "NULL pointer");
        if (ldx % 4 || ldy % 4 || !aligned16(x) || !aligned16(y))
            return arg_error(fn, "x / y must be 16-byte aligned with leading dimensions a multiple of 4");
        if (ldx > 2147483647) return arg_error(fn, "ldx too large");
        if (h % 4 == 0 && g->nnz > 0 && !aligned16(rhs)) return arg_error(fn, "rhs must be 16-byte aligned");
        if (!dispatch_dh<LaunchSpmmShared>(d, h, g, x, ldx, rhs, y, ldy, workspace,
                                           reinterpret_cast<hipStream_t>(stream)))
            return arg_error(fn, "supported: d in {32, 64, 128, 256} with h * d <= 512, h a power of two");
        return launch_status(fn);
    });
}
