// Neighbourhood ("paper-semantics") attention of U2GNN: every node attends over its own window of
// W = k+1 sampled neighbour tokens (U2GNN_tf/model_U2GNN_Sup_multi.py:14-45, where the Universal
// Transformer's batch is the node and its sequence the k+1 neighbours; restated on the torch
// encoder by feeding input_Tr.transpose(0,1)).
//
// Token rows are node-major: row n*W + s is slot s of node n; QKV [rows, 3*dp] holds the scaled
// Q (1/sqrt(d) folded in by the in-projection epilogue), K and V.  One 256-thread block per node
// stages the node's W x dp operands in LDS; the W x W scores, softmax, dropout and the products
// are fp32 VALU work (W <= 32: 17 x 17 x 384 per node is far too small for matrix cores), so
// the whole attention core of a node is one block with no HBM round trip for scores.
#include <mutex>
#include <set>
#include <utility>

#include "u2gnn_common.h"

#include <algorithm>
#include <cstdlib>

namespace {

constexpr int WIN_MAX = 32;

// rows >= n_nodes*W (padding up to rows_pad) are written as zeros by the trailing blocks
__device__ __forceinline__ bool zero_pad_rows(int64_t n_nodes, int W, int64_t rows_pad, int ncols, float *out,
                                              int64_t ldo) {
    const int64_t b = blockIdx.x;
    if (b < n_nodes) return false;
    const int64_t r0 = n_nodes * W + (b - n_nodes) * W;
    for (int64_t r = r0; r < min(r0 + W, rows_pad); ++r)
        for (int c = threadIdx.x; c < ncols; c += blockDim.x) out[r * ldo + c] = 0.f;
    return true;
}

// LDS images of the node's operands are [W][dp + 4]: the 4-float pad moves consecutive rows 4 banks
// apart, so the float4 reads of different rows at one column (the (i, j) pairs of a wave) spread
// over the banks instead of all landing on one (dp = 384 is a multiple of the bank count).
__device__ __forceinline__ int win_ld(int dp) { return dp + 4; }

// stage rows row0 .. row0+W-1 of a [rows][ld] fp32 operand (column offset col) into a [W][LD] image
__device__ __forceinline__ void win_stage(const float *src, int64_t ld, int64_t row0, int col, int W, int dp,
                                          float *img) {
    const int dq = dp / 4, LD = win_ld(dp);
    for (int e = threadIdx.x; e < W * dq; e += blockDim.x) {
        const int i = e / dq, c4 = (e - i * dq) * 4;
        *reinterpret_cast<float4 *>(img + i * LD + c4) =
            *reinterpret_cast<const float4 *>(src + (row0 + i) * ld + col + c4);
    }
}

// the same with threads t0 .. t0+nt-1 of the block (the others are busy elsewhere)
__device__ __forceinline__ void win_stage_part(const float *src, int64_t ld, int64_t row0, int col, int W, int dp,
                                               float *img, int t0, int nt) {
    const int dq = dp / 4, LD = win_ld(dp);
    for (int e = t0; e < W * dq; e += nt) {
        const int i = e / dq, c4 = (e - i * dq) * 4;
        *reinterpret_cast<float4 *>(img + i * LD + c4) =
            *reinterpret_cast<const float4 *>(src + (row0 + i) * ld + col + c4);
    }
}

// S[i][j] = A_i . B_j (i, j < W) into S[W][W+1]: one (i, j) pair per thread, float4 LDS reads,
// four partial sums by column residue combined as (s0 + s1) + (s2 + s3)
__device__ __forceinline__ void win_pair_dots(const float *A, const float *B, int W, int dp, float *S) {
#ifdef U2GNN_EXP_WIN_NODOTS   // ablation (tools/win_bench.py): scores not computed
    for (int e = threadIdx.x; e < W * W; e += blockDim.x) S[(e / W) * (W + 1) + e % W] = A[e % 4];
    return;
#endif
    const int LD4 = win_ld(dp) / 4, dq = dp / 4;
    for (int e = threadIdx.x; e < W * W; e += blockDim.x) {
        const int i = e / W, j = e - i * W;
        const float4 *a = reinterpret_cast<const float4 *>(A) + i * LD4;
        const float4 *b = reinterpret_cast<const float4 *>(B) + j * LD4;
        float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll 4
        for (int c = 0; c < dq; ++c) {
            const float4 x = a[c], y = b[c];
            s0 = fmaf(x.x, y.x, s0);
            s1 = fmaf(x.y, y.y, s1);
            s2 = fmaf(x.z, y.z, s2);
            s3 = fmaf(x.w, y.w, s3);
        }
        S[i * (W + 1) + j] = (s0 + s1) + (s2 + s3);
    }
}

// out[row0 + i][col + c] = scale * sum_j C(i, j) * M[j][c] for i < W, c < dp, with C(i, j) =
// C[i][j] (TRANS false) or C[j][i] (TRANS true) of a [W][W+1] LDS matrix.  A thread owns a float4
// column group and a block of rb <= RB rows (M read once per j for all of them); j runs in order, so
// every output is the same fp32 chain as a plain loop.  The RB coefficients of a j are loaded as one
// batch at clamped rows (rows past the block compute on a duplicate and are not stored): no
// per-row branch around an LDS read, one wait per j instead of one per coefficient.
constexpr int WIN_RB = 16;
template <bool TRANS, int RB>
__device__ __forceinline__ void win_combine_rb(const float *C, const float *M, int W, int dp, float scale, float *out,
                                               int64_t ldo, int64_t row0, int col, int nb, int rb) {
    const int dq = dp / 4, LD4 = win_ld(dp) / 4;
    const float4 *M4 = reinterpret_cast<const float4 *>(M);
    for (int e = threadIdx.x; e < dq * nb; e += blockDim.x) {
        const int c4 = e % dq, i0 = (e / dq) * rb;
        const int cnt = min(rb, W - i0);
        if (cnt <= 0) continue;
        int ri[RB];
#pragma unroll
        for (int r = 0; r < RB; ++r) ri[r] = i0 + min(r, cnt - 1);
        float4 acc[RB];
#pragma unroll
        for (int r = 0; r < RB; ++r) acc[r] = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int j = 0; j < W; ++j) {
            const float4 m = M4[j * LD4 + c4];
            float cf[RB];
#pragma unroll
            for (int r = 0; r < RB; ++r) cf[r] = TRANS ? C[j * (W + 1) + ri[r]] : C[ri[r] * (W + 1) + j];
#pragma unroll
            for (int r = 0; r < RB; ++r) {
                acc[r].x = fmaf(cf[r], m.x, acc[r].x);
                acc[r].y = fmaf(cf[r], m.y, acc[r].y);
                acc[r].z = fmaf(cf[r], m.z, acc[r].z);
                acc[r].w = fmaf(cf[r], m.w, acc[r].w);
            }
        }
#pragma unroll
        for (int r = 0; r < RB; ++r) {
            if (r < cnt) {
                float4 v = acc[r];
                if (scale != 1.f) v.x *= scale, v.y *= scale, v.z *= scale, v.w *= scale;
                *reinterpret_cast<float4 *>(out + (row0 + i0 + r) * ldo + col + 4 * c4) = v;
            }
        }
    }
}

template <bool TRANS>
__device__ __forceinline__ void win_combine(const float *C, const float *M, int W, int dp, float scale, float *out,
                                            int64_t ldo, int64_t row0, int col) {
#ifdef U2GNN_EXP_WIN_NOCOMBINE   // ablation: the products skipped, the rows still written
    for (int e = threadIdx.x; e < W * (dp / 4); e += blockDim.x)
        *reinterpret_cast<float4 *>(out + (row0 + e / (dp / 4)) * ldo + col + 4 * (e % (dp / 4))) =
            make_float4(C[0], M[0], scale, 0.f);
    return;
#endif
    const int dq = dp / 4;
    int nb = (int)blockDim.x / dq;
    const int nb_min = (W + WIN_RB - 1) / WIN_RB;
    if (nb < nb_min) nb = nb_min;
    if (nb > W) nb = W;
    const int rb = (W + nb - 1) / nb;   // block-uniform: one instantiation per launch shape
    if (rb <= 4) win_combine_rb<TRANS, 4>(C, M, W, dp, scale, out, ldo, row0, col, nb, rb);
    else if (rb <= 6) win_combine_rb<TRANS, 6>(C, M, W, dp, scale, out, ldo, row0, col, nb, rb);
    else if (rb <= 9) win_combine_rb<TRANS, 9>(C, M, W, dp, scale, out, ldo, row0, col, nb, rb);
    else if (rb <= 12) win_combine_rb<TRANS, 12>(C, M, W, dp, scale, out, ldo, row0, col, nb, rb);
    else win_combine_rb<TRANS, WIN_RB>(C, M, W, dp, scale, out, ldo, row0, col, nb, rb);
}

// forward: O_n = dropout(softmax(Qs_n K_n^T)) V_n; P_n (pre-dropout probabilities) saved.
// Two operand images (Q, K; V replaces Q once the scores exist, staged by the waves the softmax
// leaves idle): 54 KB of LDS at W = 17, dp = 384, i.e. 3 blocks per CU.
__global__ void __launch_bounds__(256) window_attn_fwd_kernel(const float *QKV, int64_t ldq, int W, int dp,
                                                              float *O, int64_t ldo, float *Psave, float p,
                                                              uint64_t seed, const uint64_t *seed_epoch, int64_t n_nodes, int64_t rows_pad) {
    seed = u2gnn_seed(seed, seed_epoch);
    if (zero_pad_rows(n_nodes, W, rows_pad, dp, O, ldo)) return;
    extern __shared__ float sm[];
    const int LD = win_ld(dp);
    float *Qs = sm, *Ks = Qs + W * LD, *S = Ks + W * LD;   // S: [W][W+1]
    float *Vs = Qs;
    const int tid = threadIdx.x;
    const int64_t n = blockIdx.x, row0 = n * W;
    win_stage(QKV, ldq, row0, 0, W, dp, Qs);
    win_stage(QKV, ldq, row0, dp, W, dp, Ks);
    __syncthreads();
    win_pair_dots(Qs, Ks, W, dp, S);
    __syncthreads();
    if (tid < 64) {
        if (tid < W) {   // row softmax, save P, keep Pd in S
            float *srow = S + tid * (W + 1);
            float m = -INFINITY;
            for (int j = 0; j < W; ++j) m = fmaxf(m, srow[j]);
            float sum = 0.f;
            for (int j = 0; j < W; ++j) {
                srow[j] = expf(srow[j] - m);
                sum += srow[j];
            }
            const float inv = 1.f / sum, ks = p > 0.f ? 1.f / (1.f - p) : 1.f;
            float *prow = Psave + (n * W + tid) * W;
            for (int j = 0; j < W; ++j) {
                const float pv = srow[j] * inv;
                prow[j] = pv;
                srow[j] = (p > 0.f) ? (u2gnn_keep(seed, (uint32_t)(row0 + tid), (uint32_t)j, p) ? pv * ks : 0.f) : pv;
            }
        }
    } else {
        win_stage_part(QKV, ldq, row0, 2 * dp, W, dp, Vs, tid - 64, blockDim.x - 64);
    }
    __syncthreads();
    win_combine<false>(S, Vs, W, dp, 1.f, O, ldo, row0, 0);
}

// Persistent forward: the same per-node maths and order (bit-identical outputs), with a block per
// LDS slot of the chip walking nodes n, n + grid, ... and the operand traffic taken off the
// critical path: the next node's Q and K are loaded into registers while this node computes, so a
// node's opening HBM latency overlaps the previous node's work (PF float4 per thread per operand:
// W * dp / 4 <= 256 * PF; V is staged during the softmax as in window_attn_fwd_kernel -- holding it
// in registers too spilled).
template <int PF>
__device__ __forceinline__ void win_regs_load(const float *src, int64_t ld, int64_t row0, int col, int W, int dq,
                                              float4 (&r)[PF]) {
#pragma unroll
    for (int q = 0; q < PF; ++q) {
        const int e = threadIdx.x + q * 256;
        r[q] = e < W * dq ? *reinterpret_cast<const float4 *>(src + (row0 + e / dq) * ld + col + (e % dq) * 4)
                          : make_float4(0.f, 0.f, 0.f, 0.f);
    }
}

template <int PF>
__device__ __forceinline__ void win_regs_store(float *img, int W, int dq, int LD, const float4 (&r)[PF]) {
#pragma unroll
    for (int q = 0; q < PF; ++q) {
        const int e = threadIdx.x + q * 256;
        if (e < W * dq) *reinterpret_cast<float4 *>(img + (e / dq) * LD + (e % dq) * 4) = r[q];
    }
}

// MINW waves per SIMD = blocks per CU (3 = the LDS bound at C4 shapes)
template <int PF, int RB, int MINW>
__global__ void __launch_bounds__(256, MINW) window_attn_fwd_pf_kernel(const float *QKV, int64_t ldq, int W, int dp,
                                                                 float *O, int64_t ldo, float *Psave, float p,
                                                                 uint64_t seed, const uint64_t *seed_epoch,
                                                                 int64_t n_nodes, int64_t rows_pad) {
    seed = u2gnn_seed(seed, seed_epoch);
    extern __shared__ float sm[];
    const int LD = win_ld(dp), dq = dp / 4;
    float *Qs = sm, *Ks = Qs + W * LD, *S = Ks + W * LD;   // S: [W][W+1]
    float *Vs = Qs;
    const int tid = threadIdx.x;
    float4 rq[PF], rk[PF];
    int64_t n = blockIdx.x;
    if (n < n_nodes) {
        win_regs_load<PF>(QKV, ldq, n * W, 0, W, dq, rq);
        win_regs_load<PF>(QKV, ldq, n * W, dp, W, dq, rk);
    }
    for (; n < n_nodes; n += gridDim.x) {
        const int64_t row0 = n * W;
        win_regs_store<PF>(Qs, W, dq, LD, rq);
        win_regs_store<PF>(Ks, W, dq, LD, rk);
        const int64_t nn = n + gridDim.x;
        if (nn < n_nodes) {   // the next node's Q, K: land during this node's work
            win_regs_load<PF>(QKV, ldq, nn * W, 0, W, dq, rq);
            win_regs_load<PF>(QKV, ldq, nn * W, dp, W, dq, rk);
        }
        __syncthreads();
        win_pair_dots(Qs, Ks, W, dp, S);
        __syncthreads();
        if (tid < 64) {
          if (tid < W) {   // row softmax, save P, keep Pd in S (as window_attn_fwd_kernel)
            float *srow = S + tid * (W + 1);
            float m = -INFINITY;
            for (int j = 0; j < W; ++j) m = fmaxf(m, srow[j]);
            float sum = 0.f;
            for (int j = 0; j < W; ++j) {
                srow[j] = expf(srow[j] - m);
                sum += srow[j];
            }
            const float inv = 1.f / sum, ks = p > 0.f ? 1.f / (1.f - p) : 1.f;
            float *prow = Psave + (n * W + tid) * W;
            for (int j = 0; j < W; ++j) {
                const float pv = srow[j] * inv;
                prow[j] = pv;
                srow[j] = (p > 0.f) ? (u2gnn_keep(seed, (uint32_t)(row0 + tid), (uint32_t)j, p) ? pv * ks : 0.f) : pv;
            }
          }
        } else {   // V over the dead Q image by the waves the softmax leaves idle
            win_stage_part(QKV, ldq, row0, 2 * dp, W, dp, Vs, tid - 64, blockDim.x - 64);
        }
        __syncthreads();
        // the combine at the one row-block width the host chose (win_combine's rule), so the
        // kernel's registers are not sized by the widest instantiation
        win_combine_rb<false, RB>(S, Vs, W, dp, 1.f, O, ldo, row0, 0, (W + RB - 1) / RB, RB);
        __syncthreads();   // the next node overwrites Qs / Ks / S
    }
    for (int64_t r = n_nodes * W + blockIdx.x; r < rows_pad; r += gridDim.x)
        for (int c = tid * 4; c < dp; c += 1024) *reinterpret_cast<float4 *>(O + r * ldo + c) = make_float4(0.f, 0.f, 0.f, 0.f);
}

// backward: from dO and the saved P -> dQKV (the Q part already multiplied by q_scale = 1/sqrt(d),
// i.e. the gradient of the in-projection's pre-scale output).  Two operand images: dO and V for
// dP; K replaces V (staged while wave 0 runs the softmax backward) for dQ beside dV; Q replaces
// dO for dK.  55 KB of LDS at W = 17, dp = 384: 2 blocks per CU.
__global__ void __launch_bounds__(256) window_attn_bwd_kernel(const float *QKV, int64_t ldq, int W, int dp,
                                                              const float *dO, int64_t ldo, const float *Psave,
                                                              float p, uint64_t seed, const uint64_t *seed_epoch, float q_scale, float *dQKV,
                                                              int64_t ldg, int64_t n_nodes, int64_t rows_pad) {
    seed = u2gnn_seed(seed, seed_epoch);
    if (zero_pad_rows(n_nodes, W, rows_pad, 3 * dp, dQKV, ldg)) return;
    extern __shared__ float sm[];
    const int LD = win_ld(dp);
    float *img0 = sm, *img1 = img0 + W * LD;
    float *Pd = img1 + W * LD, *dS = Pd + W * (W + 1);   // [W][W+1] each
    const int tid = threadIdx.x;
    const int64_t n = blockIdx.x, row0 = n * W;
    win_stage(dO, ldo, row0, 0, W, dp, img0);            // img0 = dO
    win_stage(QKV, ldq, row0, 2 * dp, W, dp, img1);      // img1 = V
    __syncthreads();
    win_pair_dots(img0, img1, W, dp, dS);   // dPd[i][j] = dO_i . V_j -> dS after the softmax backward
    __syncthreads();
    if (tid < 64) {
        if (tid < W) {
            const float *prow = Psave + (n * W + tid) * W;
            float *ds = dS + tid * (W + 1), *pd = Pd + tid * (W + 1);
            const float ks = p > 0.f ? 1.f / (1.f - p) : 1.f;
            float delta = 0.f;
            for (int j = 0; j < W; ++j) {
                const bool keep = (p > 0.f) ? u2gnn_keep(seed, (uint32_t)(row0 + tid), (uint32_t)j, p) : true;
                const float pv = prow[j];
                const float dp_ = keep ? ds[j] * ks : 0.f;   // gradient w.r.t. the pre-dropout P
                pd[j] = keep ? pv * ks : 0.f;
                ds[j] = dp_;
                delta += dp_ * pv;
            }
            for (int j = 0; j < W; ++j) ds[j] = prow[j] * (ds[j] - delta);
        }
    } else {
        win_stage_part(QKV, ldq, row0, dp, W, dp, img1, tid - 64, blockDim.x - 64);   // img1 = K
    }
    __syncthreads();
    win_combine<true>(Pd, img0, W, dp, 1.f, dQKV, ldg, row0, 2 * dp);   // dV_i = sum_j Pd[j][i] dO_j
    win_combine<false>(dS, img1, W, dp, q_scale, dQKV, ldg, row0, 0);   // dQ_i = sum_j dS[i][j] K_j
    __syncthreads();
    win_stage(QKV, ldq, row0, 0, W, dp, img0);           // img0 = Q
    __syncthreads();
    win_combine<true>(dS, img0, W, dp, 1.f, dQKV, ldg, row0, dp);       // dK_i = sum_j dS[j][i] Q_j
}

// Persistent backward (the same per-node maths and order as window_attn_bwd_kernel, bit-identical):
// the next node's dO and V are loaded into registers while this node computes and this node's Q
// while its scores are formed (K is staged beside the softmax as before; holding it in registers
// too spilled).
template <int PF, int RB, int MINW>
__global__ void __launch_bounds__(256, MINW) window_attn_bwd_pf_kernel(const float *QKV, int64_t ldq, int W, int dp,
                                                                       const float *dO, int64_t ldo,
                                                                       const float *Psave, float p, uint64_t seed,
                                                                       const uint64_t *seed_epoch, float q_scale,
                                                                       float *dQKV, int64_t ldg, int64_t n_nodes,
                                                                       int64_t rows_pad) {
    seed = u2gnn_seed(seed, seed_epoch);
    extern __shared__ float sm[];
    const int LD = win_ld(dp), dq = dp / 4;
    float *img0 = sm, *img1 = img0 + W * LD;
    float *Pd = img1 + W * LD, *dS = Pd + W * (W + 1);   // [W][W+1] each
    const int tid = threadIdx.x;
    const int nb = (W + RB - 1) / RB;
    float4 ra[PF], rv[PF], rq[PF];
    int64_t n = blockIdx.x;
    if (n < n_nodes) {
        win_regs_load<PF>(dO, ldo, n * W, 0, W, dq, ra);
        win_regs_load<PF>(QKV, ldq, n * W, 2 * dp, W, dq, rv);
    }
    for (; n < n_nodes; n += gridDim.x) {
        const int64_t row0 = n * W;
        win_regs_store<PF>(img0, W, dq, LD, ra);   // img0 = dO
        win_regs_store<PF>(img1, W, dq, LD, rv);   // img1 = V
        win_regs_load<PF>(QKV, ldq, row0, 0, W, dq, rq);   // this node's Q: lands during the dots
        const int64_t nn = n + gridDim.x;
        if (nn < n_nodes) {   // the next node's dO and V land during this node's work
            win_regs_load<PF>(dO, ldo, nn * W, 0, W, dq, ra);
            win_regs_load<PF>(QKV, ldq, nn * W, 2 * dp, W, dq, rv);
        }
        __syncthreads();
        win_pair_dots(img0, img1, W, dp, dS);
        __syncthreads();
        if (tid < 64) {
            if (tid < W) {
                const float *prow = Psave + (n * W + tid) * W;
                float *ds = dS + tid * (W + 1), *pd = Pd + tid * (W + 1);
                const float ks = p > 0.f ? 1.f / (1.f - p) : 1.f;
                float delta = 0.f;
                for (int j = 0; j < W; ++j) {
                    const bool keep = (p > 0.f) ? u2gnn_keep(seed, (uint32_t)(row0 + tid), (uint32_t)j, p) : true;
                    const float pv = prow[j];
                    const float dp_ = keep ? ds[j] * ks : 0.f;
                    pd[j] = keep ? pv * ks : 0.f;
                    ds[j] = dp_;
                    delta += dp_ * pv;
                }
                for (int j = 0; j < W; ++j) ds[j] = prow[j] * (ds[j] - delta);
            }
        } else {
            win_stage_part(QKV, ldq, row0, dp, W, dp, img1, tid - 64, blockDim.x - 64);   // img1 = K
        }
        __syncthreads();
        win_combine_rb<true, RB>(Pd, img0, W, dp, 1.f, dQKV, ldg, row0, 2 * dp, nb, RB);    // dV
        win_combine_rb<false, RB>(dS, img1, W, dp, q_scale, dQKV, ldg, row0, 0, nb, RB);   // dQ
        __syncthreads();
        win_regs_store<PF>(img0, W, dq, LD, rq);   // img0 = Q
        __syncthreads();
        win_combine_rb<true, RB>(dS, img0, W, dp, 1.f, dQKV, ldg, row0, dp, nb, RB);       // dK
        __syncthreads();   // the next node overwrites the images
    }
    for (int64_t r = n_nodes * W + blockIdx.x; r < rows_pad; r += gridDim.x)
        for (int c = tid * 4; c < 3 * dp; c += 1024)
            *reinterpret_cast<float4 *>(dQKV + r * ldg + c) = make_float4(0.f, 0.f, 0.f, 0.f);
}

inline size_t fwd_lds(int W, int dp) { return (size_t)(2 * W * (dp + 4) + W * (W + 1)) * sizeof(float); }
inline size_t bwd_lds(int W, int dp) { return (size_t)(2 * W * (dp + 4) + 2 * W * (W + 1)) * sizeof(float); }
constexpr size_t LDS_LIMIT = 160 * 1024;

// The persistent prefetching kernels run at 2 blocks per CU (measured round 2: 3 blocks per CU spill
// the forward's registers and run slower; one block per node is the generic kernel below).
constexpr int kWinPfBlocksPerCu = 2;

int cu_count() {
    static const int n = [] {
        int dev = 0, c = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            return 256;
        return c > 0 ? c : 256;
    }();
    return n;
}

// Dynamic LDS above 64 KiB must be opted into per kernel AND device (hipFuncSetAttribute acts on the current
// device): the (device, kernel) pairs already done are kept under a lock, so a second device or thread of the
// process gets its own opt-in instead of skipping it.
int lds_optin(const void *kern) {
    static std::mutex mu;
    static std::set<std::pair<int, const void *>> done;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return (int)e;
    std::lock_guard<std::mutex> lk(mu);
    if (done.count({dev, kern})) return U2GNN_OK;
    e = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_LIMIT);
    if (e != hipSuccess) return (int)e;
    done.insert({dev, kern});
    return U2GNN_OK;
}

#define U2GNN_TRY_WIN(x)                 \
    do {                                 \
        const int rc_ = (x);             \
        if (rc_ != U2GNN_OK) return rc_; \
    } while (0)

}  // namespace

extern "C" {

int u2gnn_window_attn_fwd(const float *QKV, int64_t ldq, int32_t W, int32_t dp, float *O, int64_t ldo, float *Psave,
                          float p, uint64_t seed, int64_t n_nodes, int64_t rows_pad, void *stream) {
    if (!QKV || !O || !Psave || W < 1 || W > WIN_MAX || dp < 4 || (dp & 3) || n_nodes < 1) return U2GNN_E_ARG;
    if (rows_pad < n_nodes * W || (ldq & 3) || (ldo & 3) || ldq < 3 * dp || ldo < dp) return U2GNN_E_ARG;
    if (((uintptr_t)QKV & 15) || ((uintptr_t)O & 15)) return U2GNN_E_ALIGN;
    const size_t lds = fwd_lds(W, dp);
    if (lds > LDS_LIMIT) return U2GNN_E_SHAPE;
    U2GNN_TRY_WIN(lds_optin(reinterpret_cast<const void *>(window_attn_fwd_kernel)));
    // persistent prefetching variant for the shapes it is instantiated for (C4 neighbour mode:
    // W = 17, dp = 384 -> 1632 float4 per operand = 7 per thread; win_combine's row blocks: 2 x 9)
    const int64_t elems = (int64_t)W * (dp / 4);   // float4 per operand image
    int nb = 256 / (dp / 4);
    nb = std::max(nb, (W + 15) / 16);
    nb = std::min(nb, (int)W);
    const int rb = (W + nb - 1) / nb;
    if (elems > 256 * 6 && elems <= 256 * 7 && rb == 9 && (W + 8) / 9 == nb) {
        auto kern = window_attn_fwd_pf_kernel<7, 9, kWinPfBlocksPerCu>;
        U2GNN_TRY_WIN(lds_optin(reinterpret_cast<const void *>(kern)));
        const int64_t per_cu = std::min<int64_t>(kWinPfBlocksPerCu, std::max<int64_t>(1, (int64_t)(LDS_LIMIT / lds)));
        const int64_t grid = std::min<int64_t>(n_nodes, per_cu * cu_count());
        hipLaunchKernelGGL(kern, dim3((unsigned)std::max<int64_t>(grid, 1)), dim3(256), lds, u2gnn_stream(stream), QKV,
                           ldq, W, dp, O, ldo, Psave, p, seed, u2gnn_cur_epoch(), n_nodes, rows_pad);
        return u2gnn_launch_status();
    }
    const int64_t pad_blocks = (rows_pad - n_nodes * W + W - 1) / W;
    hipLaunchKernelGGL(window_attn_fwd_kernel, dim3((unsigned)(n_nodes + pad_blocks)), dim3(256), lds,
                       u2gnn_stream(stream), QKV, ldq, W, dp, O, ldo, Psave, p, seed, u2gnn_cur_epoch(), n_nodes, rows_pad);
    return u2gnn_launch_status();
}

int u2gnn_window_attn_bwd(const float *QKV, int64_t ldq, int32_t W, int32_t dp, const float *dO, int64_t ldo,
                          const float *Psave, float p, uint64_t seed, float q_scale, float *dQKV, int64_t ldg,
                          int64_t n_nodes, int64_t rows_pad, void *stream) {
    if (!QKV || !dO || !Psave || !dQKV || W < 1 || W > WIN_MAX || dp < 4 || (dp & 3) || n_nodes < 1)
        return U2GNN_E_ARG;
    if (rows_pad < n_nodes * W || (ldq & 3) || (ldo & 3) || (ldg & 3) || ldq < 3 * dp || ldg < 3 * dp)
        return U2GNN_E_ARG;
    if (((uintptr_t)QKV & 15) || ((uintptr_t)dO & 15) || ((uintptr_t)dQKV & 15)) return U2GNN_E_ALIGN;
    const size_t lds = bwd_lds(W, dp);
    if (lds > LDS_LIMIT) return U2GNN_E_SHAPE;
    U2GNN_TRY_WIN(lds_optin(reinterpret_cast<const void *>(window_attn_bwd_kernel)));
    const int64_t elems = (int64_t)W * (dp / 4);
    int nb = 256 / (dp / 4);
    nb = std::max(nb, (W + 15) / 16);
    nb = std::min(nb, (int)W);
    const int rb = (W + nb - 1) / nb;
    if (elems > 256 * 6 && elems <= 256 * 7 && rb == 9 && (W + 8) / 9 == nb) {
        auto kern = window_attn_bwd_pf_kernel<7, 9, kWinPfBlocksPerCu>;
        U2GNN_TRY_WIN(lds_optin(reinterpret_cast<const void *>(kern)));
        const int64_t per_cu = std::min<int64_t>(kWinPfBlocksPerCu, std::max<int64_t>(1, (int64_t)(LDS_LIMIT / lds)));
        const int64_t grid = std::min<int64_t>(n_nodes, per_cu * cu_count());
        hipLaunchKernelGGL(kern, dim3((unsigned)std::max<int64_t>(grid, 1)), dim3(256), lds, u2gnn_stream(stream), QKV,
                           ldq, W, dp, dO, ldo, Psave, p, seed, u2gnn_cur_epoch(), q_scale, dQKV, ldg, n_nodes, rows_pad);
        return u2gnn_launch_status();
    }
    const int64_t pad_blocks = (rows_pad - n_nodes * W + W - 1) / W;
    hipLaunchKernelGGL(window_attn_bwd_kernel, dim3((unsigned)(n_nodes + pad_blocks)), dim3(256), lds,
                       u2gnn_stream(stream), QKV, ldq, W, dp, dO, ldo, Psave, p, seed, u2gnn_cur_epoch(), q_scale, dQKV, ldg, n_nodes,
                       rows_pad);
    return u2gnn_launch_status();
}

}  // extern "C"
