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
#include "u2gnn_common.h"

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

// forward: O_n = dropout(softmax(Qs_n K_n^T)) V_n; P_n (pre-dropout probabilities) saved
__global__ void __launch_bounds__(256) window_attn_fwd_kernel(const float *QKV, int64_t ldq, int W, int dp,
                                                              float *O, int64_t ldo, float *Psave, float p,
                                                              uint64_t seed, int64_t n_nodes, int64_t rows_pad) {
    if (zero_pad_rows(n_nodes, W, rows_pad, dp, O, ldo)) return;
    extern __shared__ float sm[];
    float *Qs = sm, *Ks = Qs + W * dp, *Vs = Ks + W * dp, *S = Vs + W * dp;   // S: [W][W+1]
    const int tid = threadIdx.x;
    const int64_t n = blockIdx.x, row0 = n * W;
    const int dq = dp / 4;
    for (int e = tid; e < W * dq; e += 256) {
        const int i = e / dq, c4 = (e - i * dq) * 4;
        const float *q = QKV + (row0 + i) * ldq + c4;
        *reinterpret_cast<float4 *>(Qs + i * dp + c4) = *reinterpret_cast<const float4 *>(q);
        *reinterpret_cast<float4 *>(Ks + i * dp + c4) = *reinterpret_cast<const float4 *>(q + dp);
        *reinterpret_cast<float4 *>(Vs + i * dp + c4) = *reinterpret_cast<const float4 *>(q + 2 * dp);
    }
    __syncthreads();
    for (int e = tid; e < W * W; e += 256) {
        const int i = e / W, j = e - i * W;
        const float *a = Qs + i * dp, *b = Ks + j * dp;
        float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
        for (int c = 0; c < dp; c += 4) {
            s0 = fmaf(a[c], b[c], s0);
            s1 = fmaf(a[c + 1], b[c + 1], s1);
            s2 = fmaf(a[c + 2], b[c + 2], s2);
            s3 = fmaf(a[c + 3], b[c + 3], s3);
        }
        S[i * (W + 1) + j] = (s0 + s1) + (s2 + s3);
    }
    __syncthreads();
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
    __syncthreads();
    for (int c = tid; c < dp; c += 256) {
        float acc[WIN_MAX];
#pragma unroll
        for (int i = 0; i < WIN_MAX; ++i) acc[i] = 0.f;
        for (int j = 0; j < W; ++j) {
            const float v = Vs[j * dp + c];
#pragma unroll
            for (int i = 0; i < WIN_MAX; ++i)
                if (i < W) acc[i] = fmaf(S[i * (W + 1) + j], v, acc[i]);
        }
#pragma unroll
        for (int i = 0; i < WIN_MAX; ++i)
            if (i < W) O[(row0 + i) * ldo + c] = acc[i];
    }
}

// backward: from dO and the saved P -> dQKV (the Q part already multiplied by q_scale = 1/sqrt(d),
// i.e. the gradient of the in-projection's pre-scale output)
__global__ void __launch_bounds__(256) window_attn_bwd_kernel(const float *QKV, int64_t ldq, int W, int dp,
                                                              const float *dO, int64_t ldo, const float *Psave,
                                                              float p, uint64_t seed, float q_scale, float *dQKV,
                                                              int64_t ldg, int64_t n_nodes, int64_t rows_pad) {
    if (zero_pad_rows(n_nodes, W, rows_pad, 3 * dp, dQKV, ldg)) return;
    extern __shared__ float sm[];
    float *Qs = sm, *Ks = Qs + W * dp, *Vs = Ks + W * dp, *dOs = Vs + W * dp;
    float *Pd = dOs + W * dp, *dS = Pd + W * (W + 1);   // [W][W+1] each
    const int tid = threadIdx.x;
    const int64_t n = blockIdx.x, row0 = n * W;
    const int dq = dp / 4;
    for (int e = tid; e < W * dq; e += 256) {
        const int i = e / dq, c4 = (e - i * dq) * 4;
        const float *q = QKV + (row0 + i) * ldq + c4;
        *reinterpret_cast<float4 *>(Qs + i * dp + c4) = *reinterpret_cast<const float4 *>(q);
        *reinterpret_cast<float4 *>(Ks + i * dp + c4) = *reinterpret_cast<const float4 *>(q + dp);
        *reinterpret_cast<float4 *>(Vs + i * dp + c4) = *reinterpret_cast<const float4 *>(q + 2 * dp);
        *reinterpret_cast<float4 *>(dOs + i * dp + c4) = *reinterpret_cast<const float4 *>(dO + (row0 + i) * ldo + c4);
    }
    __syncthreads();
    // dPd[i][j] = dO_i . V_j  -> dS (after the softmax backward below)
    for (int e = tid; e < W * W; e += 256) {
        const int i = e / W, j = e - i * W;
        const float *a = dOs + i * dp, *b = Vs + j * dp;
        float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
        for (int c = 0; c < dp; c += 4) {
            s0 = fmaf(a[c], b[c], s0);
            s1 = fmaf(a[c + 1], b[c + 1], s1);
            s2 = fmaf(a[c + 2], b[c + 2], s2);
            s3 = fmaf(a[c + 3], b[c + 3], s3);
        }
        dS[i * (W + 1) + j] = (s0 + s1) + (s2 + s3);
    }
    __syncthreads();
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
    __syncthreads();
    for (int c = tid; c < dp; c += 256) {
        for (int i = 0; i < W; ++i) {   // i = output row of dQ / key row of dK, dV
            float dq_ = 0.f, dk = 0.f, dv = 0.f;
            for (int j = 0; j < W; ++j) {
                dq_ = fmaf(dS[i * (W + 1) + j], Ks[j * dp + c], dq_);
                dk = fmaf(dS[j * (W + 1) + i], Qs[j * dp + c], dk);
                dv = fmaf(Pd[j * (W + 1) + i], dOs[j * dp + c], dv);
            }
            float *g = dQKV + (row0 + i) * ldg;
            g[c] = dq_ * q_scale;
            g[dp + c] = dk;
            g[2 * dp + c] = dv;
        }
    }
}

inline size_t fwd_lds(int W, int dp) { return (size_t)(3 * W * dp + W * (W + 1)) * sizeof(float); }
inline size_t bwd_lds(int W, int dp) { return (size_t)(4 * W * dp + 2 * W * (W + 1)) * sizeof(float); }
constexpr size_t LDS_LIMIT = 160 * 1024;

}  // namespace

extern "C" {

int u2gnn_window_attn_fwd(const float *QKV, int64_t ldq, int32_t W, int32_t dp, float *O, int64_t ldo, float *Psave,
                          float p, uint64_t seed, int64_t n_nodes, int64_t rows_pad, void *stream) {
    if (!QKV || !O || !Psave || W < 1 || W > WIN_MAX || dp < 4 || (dp & 3) || n_nodes < 1) return U2GNN_E_ARG;
    if (rows_pad < n_nodes * W || (ldq & 3) || ldq < 3 * dp) return U2GNN_E_ARG;
    const size_t lds = fwd_lds(W, dp);
    if (lds > LDS_LIMIT) return U2GNN_E_SHAPE;
    static bool attr = false;   // dynamic LDS above 64 KiB must be opted into once per kernel
    if (!attr) {
        const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(window_attn_fwd_kernel),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_LIMIT);
        if (e != hipSuccess) return (int)e;
        attr = true;
    }
    const int64_t pad_blocks = (rows_pad - n_nodes * W + W - 1) / W;
    hipLaunchKernelGGL(window_attn_fwd_kernel, dim3((unsigned)(n_nodes + pad_blocks)), dim3(256), lds,
                       u2gnn_stream(stream), QKV, ldq, W, dp, O, ldo, Psave, p, seed, n_nodes, rows_pad);
    return u2gnn_launch_status();
}

int u2gnn_window_attn_bwd(const float *QKV, int64_t ldq, int32_t W, int32_t dp, const float *dO, int64_t ldo,
                          const float *Psave, float p, uint64_t seed, float q_scale, float *dQKV, int64_t ldg,
                          int64_t n_nodes, int64_t rows_pad, void *stream) {
    if (!QKV || !dO || !Psave || !dQKV || W < 1 || W > WIN_MAX || dp < 4 || (dp & 3) || n_nodes < 1)
        return U2GNN_E_ARG;
    if (rows_pad < n_nodes * W || (ldq & 3) || (ldo & 3) || ldq < 3 * dp || ldg < 3 * dp) return U2GNN_E_ARG;
    const size_t lds = bwd_lds(W, dp);
    if (lds > LDS_LIMIT) return U2GNN_E_SHAPE;
    static bool attr = false;   // dynamic LDS above 64 KiB must be opted into once per kernel
    if (!attr) {
        const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(window_attn_bwd_kernel),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_LIMIT);
        if (e != hipSuccess) return (int)e;
        attr = true;
    }
    const int64_t pad_blocks = (rows_pad - n_nodes * W + W - 1) / W;
    hipLaunchKernelGGL(window_attn_bwd_kernel, dim3((unsigned)(n_nodes + pad_blocks)), dim3(256), lds,
                       u2gnn_stream(stream), QKV, ldq, W, dp, dO, ldo, Psave, p, seed, q_scale, dQKV, ldg, n_nodes,
                       rows_pad);
    return u2gnn_launch_status();
}

}  // extern "C"
