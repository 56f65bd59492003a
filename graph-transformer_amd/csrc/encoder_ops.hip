// Row-wise and bandwidth-bound kernels of the U2GNN encoder on gfx950:
// neighbour gather, attention softmax+dropout, post-LN forward/backward, split-K reduce /
// parameter pack, bias-gradient column sums.  All are HBM-bound streaming passes:
// one wave64 per row, coalesced lane-contiguous accesses, fp32 throughout.
#include "u2gnn_common.h"

#include <algorithm>

namespace {

// ------------------------------------------------------------------------------------------
// a2 neighbour gather (pytorch_U2GNN_Sup.py:32,39): one wave per destination row.
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) gather_rows_kernel(const float *src, int64_t ld_src, int64_t src_rows,
                                                          const int64_t *idx, int64_t idx_stride, float *dst,
                                                          int64_t ld_dst, int64_t n_rows, int64_t n_rows_pad,
                                                          int64_t d, int64_t d_pad, int32_t *err) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= n_rows_pad) return;
    float *o = dst + row * ld_dst;
    int64_t s = -1;
    if (row < n_rows) {
        s = idx[row * idx_stride];
        if (s < 0 || s >= src_rows) {
            if (lane == 0 && err) atomicExch(err, 1);
            s = -1;
        }
    }
    if (s < 0) {
        for (int64_t c = lane; c < d_pad; c += 64) o[c] = 0.f;
        return;
    }
    const float *in = src + s * ld_src;
    for (int64_t c = lane; c < d_pad; c += 64) o[c] = c < d ? in[c] : 0.f;
}

__global__ void __launch_bounds__(256) scatter_add_rows_kernel(const float *src, int64_t ld_src, const int64_t *idx,
                                                               int64_t idx_stride, float *dst, int64_t ld_dst,
                                                               int64_t n_rows, int64_t d) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= n_rows) return;
    const int64_t t = idx[row * idx_stride];
    for (int64_t c = lane; c < d; c += 64) atomicAdd(dst + t * ld_dst + c, src[row * ld_src + c]);
}

// ------------------------------------------------------------------------------------------
// split-K slab reduce + padded->real unpack; pack real->padded
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) slab_reduce_kernel(const float *src, int n_slab, int64_t slab_stride,
                                                          int64_t rows_pad, int64_t cols_pad, int64_t ld_src,
                                                          int64_t rbp, int64_t rbr, int64_t cbp, int64_t cbr,
                                                          float *dst, int64_t ld_dst, float alpha, int accumulate) {
    const int64_t total = rows_pad * cols_pad;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        const int64_t r = i / cols_pad, c = i - r * cols_pad;
        bool vr, vc;
        const int64_t rr = blk_map(r, rbp, rbr, &vr);
        const int64_t cc = blk_map(c, cbp, cbr, &vc);
        if (!vr || !vc) continue;
        float s = 0.f;
        const float *p = src + r * ld_src + c;
        for (int z = 0; z < n_slab; ++z) s += p[(int64_t)z * slab_stride];
        float *o = dst + rr * ld_dst + cc;
        *o = accumulate ? *o + alpha * s : alpha * s;
    }
}

__global__ void __launch_bounds__(256) pack_padded_kernel(const float *src, int64_t ld_src, int64_t rows_pad,
                                                          int64_t cols_pad, int64_t rbp, int64_t rbr, int64_t cbp,
                                                          int64_t cbr, float *dst, int64_t ld_dst) {
    const int64_t total = rows_pad * cols_pad;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        const int64_t r = i / cols_pad, c = i - r * cols_pad;
        bool vr, vc;
        const int64_t rr = blk_map(r, rbp, rbr, &vr);
        const int64_t cc = blk_map(c, cbp, cbr, &vc);
        dst[r * ld_dst + c] = (vr && vc) ? src[rr * ld_src + cc] : 0.f;
    }
}

// many pack jobs in one launch: the descriptors travel by value in the kernel arguments
constexpr int PACK_MAX = 32;
struct PackBatch {
    u2gnn_pack_desc d[PACK_MAX];
};

__global__ void __launch_bounds__(256) pack_multi_kernel(PackBatch pb) {
    const u2gnn_pack_desc &D = pb.d[blockIdx.y];
    const int64_t total = D.rows_pad * D.cols_pad;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        const int64_t r = i / D.cols_pad, c = i - r * D.cols_pad;
        bool vr, vc;
        const int64_t rr = blk_map(r, D.rblk_pad, D.rblk_real, &vr);
        const int64_t cc = blk_map(c, D.cblk_pad, D.cblk_real, &vc);
        D.dst[r * D.ld_dst + c] = (vr && vc) ? D.src[rr * D.ld_src + cc] : 0.f;
    }
}

// column sums, stage 1: block (64 columns x CS_ROWS rows) -> ws[chunk][col].  Each wave owns 32
// consecutive rows and keeps 8 independent loads in flight (latency, not bandwidth, bounds this).
constexpr int CS_ROWS = 128;

__global__ void __launch_bounds__(256) colsum_partial_kernel(const float *X, int64_t rows, int64_t cols_pad,
                                                             int64_t ld, float *ws) {
    __shared__ float red[4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t c = (int64_t)blockIdx.x * 64 + lane;
    const int64_t r0 = (int64_t)blockIdx.y * CS_ROWS + w * (CS_ROWS / 4);
    float s[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] = 0.f;
    if (c < cols_pad) {
#pragma unroll
        for (int i = 0; i < CS_ROWS / 4; i += 8)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int64_t r = r0 + i + j;
                if (r < rows) s[j] += X[r * ld + c];
            }
    }
    red[w][lane] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
    __syncthreads();
    if (w == 0 && c < cols_pad)
        ws[(int64_t)blockIdx.y * cols_pad + c] = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
}

__global__ void __launch_bounds__(256) colsum_final_kernel(const float *ws, int64_t n_chunks, int64_t cols_pad,
                                                           int64_t cbp, int64_t cbr, float *out, int accumulate) {
    const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (c >= cols_pad) return;
    bool v;
    const int64_t cc = blk_map(c, cbp, cbr, &v);
    if (!v) return;
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    int64_t k = 0;
    for (; k + 4 <= n_chunks; k += 4)
#pragma unroll
        for (int j = 0; j < 4; ++j) s[j] += ws[(k + j) * cols_pad + c];
    for (; k < n_chunks; ++k) s[0] += ws[k * cols_pad + c];
    const float t = (s[0] + s[1]) + (s[2] + s[3]);
    out[cc] = accumulate ? out[cc] + t : t;
}

// ------------------------------------------------------------------------------------------
// a3.2 attention probabilities: row softmax over the n_valid keys, dropout(p) on the
// probabilities (torch SDPA math path: dropout AFTER softmax, 1/(1-p) scaling).
// One 256-thread block per row; online max/sum pass, then normalise + mask pass.
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) attn_softmax_kernel(const float *S, int64_t lds, float *P, float *Pd,
                                                           int64_t ldp, int64_t rows_valid, int64_t n_valid,
                                                           int64_t n_pad, float p, uint64_t seed) {
    __shared__ float red_m[4], red_s[4];
    const int64_t row = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    float *prow = P + row * ldp;
    float *pdrow = Pd + row * ldp;
    const bool write_pd = Pd != P;
    if (row >= rows_valid) {
        for (int64_t c = tid * 4; c < n_pad; c += 1024) {
            *reinterpret_cast<float4 *>(prow + c) = make_float4(0.f, 0.f, 0.f, 0.f);
            if (write_pd) *reinterpret_cast<float4 *>(pdrow + c) = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        return;
    }
    const float *srow = S + row * lds;
    float m = -INFINITY, s = 0.f;
    for (int64_t c = tid * 4; c < n_pad; c += 1024) {
        const float4 v = *reinterpret_cast<const float4 *>(srow + c);
        const float x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (c + j < n_valid) {
                const float mn = fmaxf(m, x[j]);
                s = s * expf(m - mn) + expf(x[j] - mn);
                m = mn;
            }
        }
    }
    // combine (m, s) across the wave, then across the 4 waves
    const float mw = wave_max(m);
    s = (m == -INFINITY) ? 0.f : s * expf(m - mw);
    s = wave_sum(s);
    if (lane == 0) {
        red_m[w] = mw;
        red_s[w] = s;
    }
    __syncthreads();
    const float M = fmaxf(fmaxf(red_m[0], red_m[1]), fmaxf(red_m[2], red_m[3]));
    float tot = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) tot += red_m[i] == -INFINITY ? 0.f : red_s[i] * expf(red_m[i] - M);
    const float inv = 1.f / tot;
    const float ks = p > 0.f ? 1.f / (1.f - p) : 1.f;
    for (int64_t c = tid * 4; c < n_pad; c += 1024) {
        const float4 v = *reinterpret_cast<const float4 *>(srow + c);
        const float x[4] = {v.x, v.y, v.z, v.w};
        float e[4], ed[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            e[j] = (c + j < n_valid) ? expf(x[j] - M) * inv : 0.f;
            ed[j] = (p > 0.f) ? (u2gnn_keep(seed, (uint32_t)row, (uint32_t)(c + j), p) ? e[j] * ks : 0.f) : e[j];
        }
        *reinterpret_cast<float4 *>(prow + c) = make_float4(e[0], e[1], e[2], e[3]);
        if (write_pd) *reinterpret_cast<float4 *>(pdrow + c) = make_float4(ed[0], ed[1], ed[2], ed[3]);
    }
}

__global__ void __launch_bounds__(256) rowdot_kernel(const float *A, int64_t lda, const float *B, int64_t ldb,
                                                     float *out, int64_t rows, int64_t cols) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= rows) return;
    float s = 0.f;
    for (int64_t c = lane; c < cols; c += 64) s += A[row * lda + c] * B[row * ldb + c];
    s = wave_sum(s);
    if (lane == 0) out[row] = s;
}

// ------------------------------------------------------------------------------------------
// a3.3/a3.4 post-LN (eps 1e-5). One wave per row, row cached in registers (d_pad <= 1024).
// ------------------------------------------------------------------------------------------
constexpr int LN_MAXV = 16;  // d_pad / 64 upper bound

__global__ void __launch_bounds__(256) layernorm_fwd_kernel(const float *Z, int64_t ldz, const float *gamma,
                                                            const float *beta, float *Y, int64_t ldy, float *mean,
                                                            float *rstd, int64_t rows_valid, int64_t rows_pad,
                                                            int64_t d, int64_t d_pad, float eps) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= rows_pad) return;
    float *y = Y + row * ldy;
    if (row >= rows_valid) {
        for (int64_t c = lane; c < d_pad; c += 64) y[c] = 0.f;
        if (lane == 0) {
            mean[row] = 0.f;
            rstd[row] = 0.f;
        }
        return;
    }
    const float *z = Z + row * ldz;
    float v[LN_MAXV];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i) {
        const int64_t c = lane + 64 * i;
        v[i] = (c < d) ? z[c] : 0.f;
        s += v[i];
    }
    const float mu = wave_sum(s) / (float)d;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i) {
        const int64_t c = lane + 64 * i;
        const float t = (c < d) ? v[i] - mu : 0.f;
        q += t * t;
    }
    const float var = wave_sum(q) / (float)d;
    const float rs = rsqrtf(var + eps);
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i) {
        const int64_t c = lane + 64 * i;
        if (c < d)
            y[c] = (v[i] - mu) * rs * gamma[c] + beta[c];
        else if (c < d_pad)
            y[c] = 0.f;
    }
    if (lane == 0) {
        mean[row] = mu;
        rstd[row] = rs;
    }
}

// LN backward, row part: one wave per row (4 rows per block, fully parallel over rows).
__global__ void __launch_bounds__(256) layernorm_bwd_kernel(const float *dY, int64_t ldy, const float *Z, int64_t ldz,
                                                            const float *mean, const float *rstd, const float *gamma,
                                                            float *dZ, int64_t lddz, float *dZd, int64_t lddrop,
                                                            float p, uint64_t seed, int64_t rows_valid,
                                                            int64_t rows_pad, int64_t d, int64_t d_pad) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= rows_pad) return;
    float *dz = dZ + row * lddz;
    float *dzd = dZd ? dZd + row * lddrop : nullptr;
    if (row >= rows_valid) {
        for (int64_t c = lane; c < d_pad; c += 64) {
            dz[c] = 0.f;
            if (dzd) dzd[c] = 0.f;
        }
        return;
    }
    const float ks = p > 0.f ? 1.f / (1.f - p) : 1.f;
    const float mu = mean[row], rs = rstd[row];
    const float *dy = dY + row * ldy;
    const float *z = Z + row * ldz;
    float xh[LN_MAXV], g[LN_MAXV];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i) {
        const int64_t c = lane + 64 * i;
        if (c < d) {
            xh[i] = (z[c] - mu) * rs;
            g[i] = dy[c] * gamma[c];
        } else {
            xh[i] = 0.f;
            g[i] = 0.f;
        }
        s1 += g[i];
        s2 += g[i] * xh[i];
    }
    const float m1 = wave_sum(s1) / (float)d;
    const float m2 = wave_sum(s2) / (float)d;
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i) {
        const int64_t c = lane + 64 * i;
        if (c < d) {
            const float v = rs * (g[i] - m1 - xh[i] * m2);
            dz[c] = v;
            if (dzd) dzd[c] = (p > 0.f) ? (u2gnn_keep(seed, (uint32_t)row, (uint32_t)c, p) ? v * ks : 0.f) : v;
        } else if (c < d_pad) {
            dz[c] = 0.f;
            if (dzd) dzd[c] = 0.f;
        }
    }
}

// LN backward, column part: per 128-row chunk, sums over rows of dY*xhat (dgamma), dY (dbeta)
// and dZd (the bias gradient of the dropout branch feeding this LN) -> ws[chunk][3][d_pad].
__global__ void __launch_bounds__(256) ln_colstats_kernel(const float *dY, int64_t ldy, const float *Z, int64_t ldz,
                                                          const float *mean, const float *rstd, const float *dZd,
                                                          int64_t lddrop, int64_t rows, int64_t d, int64_t d_pad,
                                                          float *ws) {
    __shared__ float red[4][3][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t c = (int64_t)blockIdx.x * 64 + lane;
    const int64_t r0 = (int64_t)blockIdx.y * CS_ROWS + w * (CS_ROWS / 4);
    float sg[4] = {0.f, 0.f, 0.f, 0.f}, sb[4] = {0.f, 0.f, 0.f, 0.f}, sd[4] = {0.f, 0.f, 0.f, 0.f};
    if (c < d) {
#pragma unroll
        for (int i = 0; i < CS_ROWS / 4; i += 4)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int64_t r = r0 + i + j;
                if (r < rows) {
                    const float dy = dY[r * ldy + c];
                    sg[j] += dy * ((Z[r * ldz + c] - mean[r]) * rstd[r]);
                    sb[j] += dy;
                    if (dZd) sd[j] += dZd[r * lddrop + c];
                }
            }
    }
    red[w][0][lane] = (sg[0] + sg[1]) + (sg[2] + sg[3]);
    red[w][1][lane] = (sb[0] + sb[1]) + (sb[2] + sb[3]);
    red[w][2][lane] = (sd[0] + sd[1]) + (sd[2] + sd[3]);
    __syncthreads();
    if (w < 3 && c < d_pad)
        ws[((int64_t)blockIdx.y * 3 + w) * d_pad + c] = red[0][w][lane] + red[1][w][lane] + red[2][w][lane] +
                                                      red[3][w][lane];
}

__global__ void __launch_bounds__(256) ln_param_reduce_kernel(const float *ws, int64_t n_chunks, int64_t d,
                                                              int64_t d_pad, float *dgamma, float *dbeta, float *dbias) {
    const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (c >= d) return;
    float a[4] = {0.f, 0.f, 0.f, 0.f};
    float b[4] = {0.f, 0.f, 0.f, 0.f};
    float e[4] = {0.f, 0.f, 0.f, 0.f};
    int64_t k = 0;
    for (; k + 4 <= n_chunks; k += 4)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float *q = ws + (k + j) * 3 * d_pad + c;
            a[j] += q[0];
            b[j] += q[d_pad];
            e[j] += q[2 * d_pad];
        }
    for (; k < n_chunks; ++k) {
        const float *q = ws + k * 3 * d_pad + c;
        a[0] += q[0];
        b[0] += q[d_pad];
        e[0] += q[2 * d_pad];
    }
    dgamma[c] = (a[0] + a[1]) + (a[2] + a[3]);
    dbeta[c] = (b[0] + b[1]) + (b[2] + b[3]);
    if (dbias) dbias[c] = (e[0] + e[1]) + (e[2] + e[3]);
}

__global__ void __launch_bounds__(256) dropout_mask_kernel(uint64_t seed, int64_t rows, int64_t cols, float p,
                                                           uint8_t *out) {
    const int64_t total = rows * cols;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        const int64_t r = i / cols, c = i - r * cols;
        out[i] = u2gnn_keep(seed, (uint32_t)r, (uint32_t)c, p) ? 1 : 0;
    }
}

__global__ void __launch_bounds__(256) dropout_kernel(const float *X, int64_t ldx, float *Y, int64_t ldy, int64_t rows,
                                                      int64_t cols, float p, uint64_t seed) {
    const int64_t total = rows * cols;
    const float ks = 1.f / (1.f - p);
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        const int64_t r = i / cols, c = i - r * cols;
        const float v = X[r * ldx + c];
        Y[r * ldy + c] = u2gnn_keep(seed, (uint32_t)r, (uint32_t)c, p) ? v * ks : 0.f;
    }
}

inline unsigned grid_for(int64_t n, int64_t per_block, int64_t cap = 8192) {
    int64_t g = (n + per_block - 1) / per_block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}

}  // namespace

extern "C" {

int u2gnn_gather_rows(const float *src, int64_t ld_src, int64_t src_rows, const int64_t *idx, int64_t idx_stride,
                      float *dst, int64_t ld_dst, int64_t n_rows, int64_t n_rows_pad, int64_t d, int64_t d_pad,
                      int32_t *err, void *stream) {
    if (!dst || (n_rows > 0 && (!src || !idx)) || n_rows > n_rows_pad || d > d_pad) return U2GNN_E_ARG;
    if (n_rows_pad == 0) return U2GNN_OK;
    hipLaunchKernelGGL(gather_rows_kernel, dim3(grid_for(n_rows_pad, 4, 1 << 30)), dim3(256), 0, u2gnn_stream(stream),
                       src, ld_src, src_rows, idx, idx_stride, dst, ld_dst, n_rows, n_rows_pad, d, d_pad, err);
    return u2gnn_launch_status();
}

int u2gnn_scatter_add_rows(const float *src, int64_t ld_src, const int64_t *idx, int64_t idx_stride, float *dst,
                           int64_t ld_dst, int64_t n_rows, int64_t d, void *stream) {
    if (n_rows == 0) return U2GNN_OK;
    if (!src || !idx || !dst) return U2GNN_E_ARG;
    hipLaunchKernelGGL(scatter_add_rows_kernel, dim3(grid_for(n_rows, 4, 1 << 30)), dim3(256), 0,
                       u2gnn_stream(stream), src, ld_src, idx, idx_stride, dst, ld_dst, n_rows, d);
    return u2gnn_launch_status();
}

int u2gnn_slab_reduce(const float *src, int32_t n_slab, int64_t slab_stride, int64_t rows_pad, int64_t cols_pad,
                      int64_t ld_src, int64_t rblk_pad, int64_t rblk_real, int64_t cblk_pad, int64_t cblk_real,
                      float *dst, int64_t ld_dst, float alpha, int32_t accumulate, void *stream) {
    if (!src || !dst || n_slab < 1 || rblk_pad < 1 || cblk_pad < 1) return U2GNN_E_ARG;
    hipLaunchKernelGGL(slab_reduce_kernel, dim3(grid_for(rows_pad * cols_pad, 256)), dim3(256), 0,
                       u2gnn_stream(stream), src, n_slab, slab_stride, rows_pad, cols_pad, ld_src, rblk_pad, rblk_real,
                       cblk_pad, cblk_real, dst, ld_dst, alpha, accumulate);
    return u2gnn_launch_status();
}

int u2gnn_pack_padded(const float *src, int64_t ld_src, int64_t rows_pad, int64_t cols_pad, int64_t rblk_pad,
                      int64_t rblk_real, int64_t cblk_pad, int64_t cblk_real, float *dst, int64_t ld_dst,
                      void *stream) {
    if (!src || !dst || rblk_pad < 1 || cblk_pad < 1) return U2GNN_E_ARG;
    hipLaunchKernelGGL(pack_padded_kernel, dim3(grid_for(rows_pad * cols_pad, 256)), dim3(256), 0,
                       u2gnn_stream(stream), src, ld_src, rows_pad, cols_pad, rblk_pad, rblk_real, cblk_pad, cblk_real,
                       dst, ld_dst);
    return u2gnn_launch_status();
}

int u2gnn_pack_padded_multi(const u2gnn_pack_desc *descs, int32_t n, void *stream) {
    if (n < 0 || (n && !descs)) return U2GNN_E_ARG;
    for (int32_t o = 0; o < n; o += PACK_MAX) {
        PackBatch pb;
        const int32_t m = n - o < PACK_MAX ? n - o : PACK_MAX;
        int64_t biggest = 1;
        for (int32_t i = 0; i < m; ++i) {
            pb.d[i] = descs[o + i];
            if (!pb.d[i].src || !pb.d[i].dst || pb.d[i].rblk_pad < 1 || pb.d[i].cblk_pad < 1) return U2GNN_E_ARG;
            biggest = std::max<int64_t>(biggest, pb.d[i].rows_pad * pb.d[i].cols_pad);
        }
        hipLaunchKernelGGL(pack_multi_kernel, dim3(grid_for(biggest, 256, 2048), (unsigned)m), dim3(256), 0,
                           u2gnn_stream(stream), pb);
    }
    return u2gnn_launch_status();
}

int u2gnn_colsum(const float *X, int64_t rows, int64_t cols_pad, int64_t ld, int64_t cblk_pad, int64_t cblk_real,
                 float *out, int32_t accumulate, float *ws, void *stream) {
    if (!X || !out || !ws || cblk_pad < 1) return U2GNN_E_ARG;
    const int64_t chunks = (rows + CS_ROWS - 1) / CS_ROWS;
    hipStream_t st = u2gnn_stream(stream);
    hipLaunchKernelGGL(colsum_partial_kernel, dim3((unsigned)((cols_pad + 63) / 64), (unsigned)(chunks > 0 ? chunks : 1)),
                       dim3(256), 0, st, X, rows, cols_pad, ld, ws);
    hipLaunchKernelGGL(colsum_final_kernel, dim3(grid_for(cols_pad, 256, 1 << 30)), dim3(256), 0, st, ws,
                       chunks > 0 ? chunks : 1, cols_pad, cblk_pad, cblk_real, out, accumulate);
    return u2gnn_launch_status();
}

int u2gnn_attn_softmax_fwd(const float *S, int64_t lds, float *P, float *Pd, int64_t ldp, int64_t rows_valid,
                           int64_t rows_pad, int64_t n_valid, int64_t n_pad, float p, uint64_t seed, void *stream) {
    if (!S || !P || !Pd || (n_pad & 3) || (lds & 3) || (ldp & 3) || n_valid > n_pad || n_valid < 1) return U2GNN_E_ARG;
    if (Pd == P && p > 0.f) return U2GNN_E_ARG;
    hipLaunchKernelGGL(attn_softmax_kernel, dim3((unsigned)rows_pad), dim3(256), 0, u2gnn_stream(stream), S, lds, P,
                       Pd, ldp, rows_valid, n_valid, n_pad, p, seed);
    return u2gnn_launch_status();
}

int u2gnn_rowdot(const float *A, int64_t lda, const float *B, int64_t ldb, float *out, int64_t rows, int64_t cols,
                 void *stream) {
    if (!A || !B || !out) return U2GNN_E_ARG;
    if (rows == 0) return U2GNN_OK;
    hipLaunchKernelGGL(rowdot_kernel, dim3(grid_for(rows, 4, 1 << 30)), dim3(256), 0, u2gnn_stream(stream), A, lda, B,
                       ldb, out, rows, cols);
    return u2gnn_launch_status();
}

int u2gnn_layernorm_fwd(const float *Z, int64_t ldz, const float *gamma, const float *beta, float *Y, int64_t ldy,
                        float *mean, float *rstd, int64_t rows_valid, int64_t rows_pad, int64_t d, int64_t d_pad,
                        float eps, void *stream) {
    if (!Z || !gamma || !beta || !Y || !mean || !rstd || d < 1 || d > d_pad || d_pad > LN_MAXV * 64)
        return U2GNN_E_ARG;
    hipLaunchKernelGGL(layernorm_fwd_kernel, dim3(grid_for(rows_pad, 4, 1 << 30)), dim3(256), 0, u2gnn_stream(stream),
                       Z, ldz, gamma, beta, Y, ldy, mean, rstd, rows_valid, rows_pad, d, d_pad, eps);
    return u2gnn_launch_status();
}

int u2gnn_layernorm_bwd(const float *dY, int64_t ldy, const float *Z, int64_t ldz, const float *mean,
                        const float *rstd, const float *gamma, float *dZ, int64_t lddz, float *dZdrop, int64_t lddrop,
                        float p, uint64_t seed, int64_t rows_valid, int64_t rows_pad, int64_t d, int64_t d_pad,
                        void *stream) {
    if (!dY || !Z || !mean || !rstd || !gamma || !dZ || d < 1 || d > d_pad || d_pad > LN_MAXV * 64)
        return U2GNN_E_ARG;
    hipLaunchKernelGGL(layernorm_bwd_kernel, dim3(grid_for(rows_pad, 4, 1 << 30)), dim3(256), 0, u2gnn_stream(stream),
                       dY, ldy, Z, ldz, mean, rstd, gamma, dZ, lddz, dZdrop, lddrop, p, seed, rows_valid, rows_pad, d,
                       d_pad);
    return u2gnn_launch_status();
}

int u2gnn_layernorm_bwd_params(const float *dY, int64_t ldy, const float *Z, int64_t ldz, const float *mean,
                               const float *rstd, const float *dZdrop, int64_t lddrop, int64_t rows_valid, int64_t d,
                               int64_t d_pad, float *ws, float *dgamma, float *dbeta, float *dbias, void *stream) {
    if (!dY || !Z || !mean || !rstd || !ws || !dgamma || !dbeta || d < 1 || d > d_pad) return U2GNN_E_ARG;
    if (dbias && !dZdrop) return U2GNN_E_ARG;
    const int64_t chunks = rows_valid > 0 ? (rows_valid + CS_ROWS - 1) / CS_ROWS : 1;
    hipStream_t st = u2gnn_stream(stream);
    hipLaunchKernelGGL(ln_colstats_kernel, dim3((unsigned)((d + 63) / 64), (unsigned)chunks), dim3(256), 0, st, dY,
                       ldy, Z, ldz, mean, rstd, dbias ? dZdrop : nullptr, lddrop, rows_valid, d, d_pad, ws);
    hipLaunchKernelGGL(ln_param_reduce_kernel, dim3(grid_for(d, 256, 1 << 30)), dim3(256), 0, st, ws, chunks, d, d_pad,
                       dgamma, dbeta, dbias);
    return u2gnn_launch_status();
}

int u2gnn_dropout(const float *X, int64_t ldx, float *Y, int64_t ldy, int64_t rows, int64_t cols, float p,
                  uint64_t seed, void *stream) {
    if (!X || !Y || p < 0.f || p >= 1.f) return U2GNN_E_ARG;
    if (rows * cols == 0) return U2GNN_OK;
    hipLaunchKernelGGL(dropout_kernel, dim3(grid_for(rows * cols, 256)), dim3(256), 0, u2gnn_stream(stream), X, ldx, Y,
                       ldy, rows, cols, p, seed);
    return u2gnn_launch_status();
}

int u2gnn_dropout_mask(uint64_t seed, int64_t rows, int64_t cols, float p, uint8_t *out, void *stream) {
    if (!out) return U2GNN_E_ARG;
    hipLaunchKernelGGL(dropout_mask_kernel, dim3(grid_for(rows * cols, 256)), dim3(256), 0, u2gnn_stream(stream), seed,
                       rows, cols, p, out);
    return u2gnn_launch_status();
}

}  // extern "C"
