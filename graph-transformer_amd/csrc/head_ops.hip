// Graph-level kernels of U2GNN on gfx950: sum pooling (+dropout), the per-layer linear
// head, the label-smoothed cross-entropy, the fused clip_grad_norm_ + Adam sweep, and the
// sampled-softmax loss of the unsupervised model.
#include "u2gnn_common.h"

#include <atomic>

// seed epoch of each device (u2gnn_set_seed_epoch records it for the calling thread's current device); every
// dropout-drawing launch passes the entry of the device it is issued on (the current device: the streams the
// callers pass belong to it), so two devices driven from one process keep separate epochs
namespace {
constexpr int kMaxDevices = 64;
std::atomic<const uint64_t *> g_epoch[kMaxDevices];
int current_device() {
    int d = -1;
    return hipGetDevice(&d) == hipSuccess && d >= 0 && d < kMaxDevices ? d : -1;
}
}  // namespace

const uint64_t *u2gnn_cur_epoch() {
    const int d = current_device();
    return d < 0 ? nullptr : g_epoch[d].load(std::memory_order_acquire);
}

namespace {

// ------------------------------------------------------------------------------------------
// a5/a6 pooling: torch.spmm(graph_pool, output_Tr) with graph_pool in CSR form
// (pytorch_U2GNN_Sup.py:41) followed by dropout (:42).  Block = one graph x 64 columns.
// ------------------------------------------------------------------------------------------
// block = (graph, 64-column chunk); POOL_WAVES waves split the graph's rows, each with 4 rows' index,
// weight and feature loads in flight (the per-row chain colidx -> X is latency-bound: a COLLAB graph's
// ~75 rows over 4 waves of 1 load each took 14 us per C4 launch)
constexpr int POOL_WAVES = 8;

__global__ void __launch_bounds__(64 * POOL_WAVES) pool_fwd_kernel(const float *X, int64_t ldx, const int64_t *rowptr,
                                                                   const int64_t *colidx, const float *vals, float *G,
                                                                   int64_t ldg, int64_t d, float p, uint64_t seed,
                                                                   const uint64_t *seed_epoch) {
    seed = u2gnn_seed(seed, seed_epoch);
    __shared__ float red[POOL_WAVES][64];
    const int64_t b = blockIdx.x;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t e0 = rowptr[b], e1 = rowptr[b + 1];
    const int64_t c = (int64_t)blockIdx.y * 64 + lane;
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    if (c < d) {
        constexpr int NW = POOL_WAVES;
        int64_t e = e0 + w;
        for (; e + 3 * NW < e1; e += 4 * NW) {
            int64_t r[4];
            float v[4], x[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) r[j] = colidx[e + j * NW], v[j] = vals[e + j * NW];
#pragma unroll
            for (int j = 0; j < 4; ++j) x[j] = X[r[j] * ldx + c];
#pragma unroll
            for (int j = 0; j < 4; ++j) s[j] += v[j] * x[j];
        }
        for (; e < e1; e += NW) s[0] += vals[e] * X[colidx[e] * ldx + c];
    }
    red[w][lane] = (s[0] + s[1]) + (s[2] + s[3]);
    __syncthreads();
    if (w == 0 && c < d) {
        float v = 0.f;
#pragma unroll
        for (int q = 0; q < POOL_WAVES; ++q) v += red[q][lane];
        if (p > 0.f) v = u2gnn_keep(seed, (uint32_t)b, (uint32_t)c, p) ? v * (1.f / (1.f - p)) : 0.f;
        G[b * ldg + c] = v;
    }
}

__global__ void __launch_bounds__(256) pool_bwd_kernel(const float *dGd, int64_t ldg, const int64_t *rowptr,
                                                       const int64_t *colidx, const float *vals, float *dX,
                                                       int64_t ldx, int64_t d, float p, uint64_t seed, const uint64_t *seed_epoch) {
    seed = u2gnn_seed(seed, seed_epoch);
    // block = (graph, row slice, 64-column chunk); one atomic per (row, column)
    const int64_t b = blockIdx.x;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t e0 = rowptr[b], e1 = rowptr[b + 1];
    {
        const int64_t c = (int64_t)blockIdx.z * 64 + lane;
        if (c >= d) return;
        float g = dGd[b * ldg + c];
        if (p > 0.f) g = u2gnn_keep(seed, (uint32_t)b, (uint32_t)c, p) ? g * (1.f / (1.f - p)) : 0.f;
        for (int64_t e = e0 + (int64_t)blockIdx.y * 4 + w; e < e1; e += (int64_t)gridDim.y * 4)
            atomicAdd(dX + colidx[e] * ldx + c, vals[e] * g);
    }
}

// Pool backward for block-row pools (every row index appears once in colidx[0, N), N = rowptr[B]):
// plain stores instead of atomics into a zero-filled buffer.  Blocks x < B write their graph's rows,
// columns >= d as 0; blocks x >= B zero the padding rows [N, rows_pad), one row per wave.
__global__ void __launch_bounds__(256) pool_bwd_rows_kernel(const float *dGd, int64_t ldg, const int64_t *rowptr,
                                                            const int64_t *colidx, const float *vals, float *dX,
                                                            int64_t ldx, int64_t B, int64_t d, int64_t d_pad, int64_t N,
                                                            int64_t rows_pad, float p, uint64_t seed,
                                                            const uint64_t *seed_epoch) {
    seed = u2gnn_seed(seed, seed_epoch);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t c = (int64_t)blockIdx.z * 64 + lane;
    if (c >= d_pad) return;
    const int64_t waves = (int64_t)gridDim.y * 4;
    if ((int64_t)blockIdx.x < B) {
        const int64_t b = blockIdx.x;
        const int64_t e0 = rowptr[b], e1 = rowptr[b + 1];
        float g = 0.f;
        if (c < d) {
            g = dGd[b * ldg + c];
            if (p > 0.f) g = u2gnn_keep(seed, (uint32_t)b, (uint32_t)c, p) ? g * (1.f / (1.f - p)) : 0.f;
        }
        for (int64_t e = e0 + (int64_t)blockIdx.y * 4 + w; e < e1; e += waves)
            dX[colidx[e] * ldx + c] = c < d ? vals[e] * g : 0.f;
    } else {
        const int64_t r = N + ((int64_t)blockIdx.x - B) * waves + (int64_t)blockIdx.y * 4 + w;
        if (r < rows_pad) dX[r * ldx + c] = 0.f;
    }
}

// head: scores[b, k] (+)= G[b,:] . W[k,:] + bias[k];  one wave per (b, k)
__global__ void __launch_bounds__(256) head_fwd_kernel(const float *G, int64_t ldg, const float *W, const float *bias,
                                                       float *scores, int64_t B, int64_t C, int64_t d, int accumulate) {
    const int64_t o = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (o >= B * C) return;
    const int64_t b = o / C, k = o - b * C;
    float s = 0.f;
    for (int64_t j = lane; j < d; j += 64) s += G[b * ldg + j] * W[k * d + j];
    s = wave_sum(s);
    if (lane == 0) scores[o] = (accumulate ? scores[o] : 0.f) + s + bias[k];
}

// head backward, one thread per output element: dG[b, j] (B*d), dW[k, j] (C*d), db[k] (C)
__global__ void __launch_bounds__(256) head_bwd_kernel(const float *dS, const float *G, int64_t ldg, const float *W,
                                                       float *dG, int64_t lddg, float *dW, float *db, int64_t B,
                                                       int64_t C, int64_t d, int accumulate) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t < B * d) {
        const int64_t b = t / d, j = t - b * d;
        float s = 0.f;
        for (int64_t k = 0; k < C; ++k) s += dS[b * C + k] * W[k * d + j];
        dG[b * lddg + j] = s;
    } else if (t < B * d + C * d) {
        const int64_t u = t - B * d, k = u / d, j = u - k * d;
        float s[4] = {0.f, 0.f, 0.f, 0.f};
        int64_t b = 0;
        for (; b + 16 <= B; b += 16) {   // 16 rows' loads in flight; s[q] still sums b = q mod 4 in order
            float x[16], y[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) x[q] = dS[(b + q) * C + k], y[q] = G[(b + q) * ldg + j];
#pragma unroll
            for (int q = 0; q < 16; ++q) s[q & 3] += x[q] * y[q];
        }
        for (; b + 4 <= B; b += 4)
#pragma unroll
            for (int q = 0; q < 4; ++q) s[q] += dS[(b + q) * C + k] * G[(b + q) * ldg + j];
        for (; b < B; ++b) s[0] += dS[b * C + k] * G[b * ldg + j];
        const float v = (s[0] + s[1]) + (s[2] + s[3]);
        dW[k * d + j] = accumulate ? dW[k * d + j] + v : v;
    } else if (t < B * d + C * d + C) {
        const int64_t k = t - B * d - C * d;
        float s = 0.f;
        for (int64_t b = 0; b < B; ++b) s += dS[b * C + k];
        db[k] = accumulate ? db[k] + s : s;
    }
}

// a7: label smoothing (0.9 / 0.1/(C-1)) + mean soft cross-entropy; single block.
__global__ void __launch_bounds__(256) smoothed_ce_kernel(const float *scores, const int64_t *labels, int64_t B,
                                                          int64_t C, float smoothing, float *loss, float *dscores) {
    __shared__ float red[256];
    float acc = 0.f;
    const float off = smoothing / (float)(C - 1), on = 1.f - smoothing;
    for (int64_t b = threadIdx.x; b < B; b += 256) {
        const float *s = scores + b * C;
        float m = -INFINITY;
        for (int64_t k = 0; k < C; ++k) m = fmaxf(m, s[k]);
        float z = 0.f;
        for (int64_t k = 0; k < C; ++k) z += expf(s[k] - m);
        const float lz = logf(z);
        const int64_t y = labels[b];
        for (int64_t k = 0; k < C; ++k) {
            const float t = (k == y) ? on : off;
            const float ls = s[k] - m - lz;
            acc += -t * ls;
            dscores[b * C + k] = (expf(ls) - t) / (float)B;
        }
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) loss[0] = red[0] / (float)B;
}

// ------------------------------------------------------------------------------------------
// a9: clip_grad_norm_ + Adam over one flat fp32 buffer
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) sqnorm_partial_kernel(const float *g, int64_t n, double *ws) {
    __shared__ double red[4];
    double s = 0.0;
    const int64_t n4 = n >> 2;
    const float4 *g4 = reinterpret_cast<const float4 *>(g);
    // 4 float4 loads in flight per thread (one at a time left the 41 MB C5 sweep at 3 TB/s)
    const int64_t stride = (int64_t)gridDim.x * 256;
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + 3 * stride < n4; i += 4 * stride) {
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = g4[i + u * stride];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            s += (double)v[u].x * v[u].x + (double)v[u].y * v[u].y + (double)v[u].z * v[u].z + (double)v[u].w * v[u].w;
    }
    for (; i < n4; i += stride) {
        const float4 v = g4[i];
        s += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
    }
    if (blockIdx.x == 0)
        for (int64_t i = (n4 << 2) + threadIdx.x; i < n; i += 256) s += (double)g[i] * g[i];
    s = wave_sum_d(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) ws[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ void __launch_bounds__(256) sqnorm_final_kernel(const double *ws, int nb, float *out) {
    __shared__ double red[4];
    double s = 0.0;
    for (int i = threadIdx.x; i < nb; i += 256) s += ws[i];
    s = wave_sum_d(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) out[0] = (float)(red[0] + red[1] + red[2] + red[3]);
}

// the element update of both Adam kernels; 16-byte loads of all four streams when the buffers allow
// (one float per thread kept ~16 KB in flight per CU: C5's 326 MB sweep ran at 6 TB/s), the same
// per-element arithmetic either way
__device__ __forceinline__ void adam_sweep(float *param, const float *grad, float *m, float *v, int64_t n, float coef,
                                           float b2, float w1, float w2, float eps, float step_size, float bc2_sqrt) {
    const bool vec = ((reinterpret_cast<uintptr_t>(param) | reinterpret_cast<uintptr_t>(grad) |
                       reinterpret_cast<uintptr_t>(m) | reinterpret_cast<uintptr_t>(v)) & 15) == 0;
    const int64_t n4 = vec ? n >> 2 : 0;
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < n4; q += stride) {
        const float4 g4 = reinterpret_cast<const float4 *>(grad)[q], p4 = reinterpret_cast<const float4 *>(param)[q];
        const float4 m4 = reinterpret_cast<const float4 *>(m)[q], v4 = reinterpret_cast<const float4 *>(v)[q];
        const float gv[4] = {g4.x, g4.y, g4.z, g4.w}, pv[4] = {p4.x, p4.y, p4.z, p4.w};
        const float mv[4] = {m4.x, m4.y, m4.z, m4.w}, vv[4] = {v4.x, v4.y, v4.z, v4.w};
        float mo[4], vo[4], po[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float g = gv[k] * coef;
            mo[k] = mv[k] + w1 * (g - mv[k]);
            vo[k] = vv[k] * b2 + w2 * g * g;
            const float denom = sqrtf(vo[k]) / bc2_sqrt + eps;
            po[k] = pv[k] - step_size * (mo[k] / denom);
        }
        reinterpret_cast<float4 *>(m)[q] = make_float4(mo[0], mo[1], mo[2], mo[3]);
        reinterpret_cast<float4 *>(v)[q] = make_float4(vo[0], vo[1], vo[2], vo[3]);
        reinterpret_cast<float4 *>(param)[q] = make_float4(po[0], po[1], po[2], po[3]);
    }
    for (int64_t i = 4 * n4 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        const float g = grad[i] * coef;
        const float mi = m[i] + w1 * (g - m[i]);
        const float vi = v[i] * b2 + w2 * g * g;
        m[i] = mi;
        v[i] = vi;
        const float denom = sqrtf(vi) / bc2_sqrt + eps;
        param[i] = param[i] - step_size * (mi / denom);
    }
}

// The clip coefficient.  With sqnorm partials (SqParts, ABI v11 u2gnn_adam_sq / u2gnn_adam_dev_sq) every block
// folds the sqnorm_partial_kernel outputs exactly as sqnorm_final_kernel does (same order, same bits) and
// block 0 also stores the total: the separate one-block launch goes.
struct SqParts {
    const double *parts;   // nullptr: use sqnorm
    int nb;
    float *out;
};

__device__ __forceinline__ float clip_coef(const float *sqnorm, const SqParts &sp, float max_norm) {
    if (sp.parts) {
        __shared__ double red[4];
        double s = 0.0;
        for (int i = threadIdx.x; i < sp.nb; i += 256) s += sp.parts[i];
        s = wave_sum_d(s);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
        __syncthreads();
        const float sq = (float)(red[0] + red[1] + red[2] + red[3]);
        if (blockIdx.x == 0 && threadIdx.x == 0 && sp.out) sp.out[0] = sq;
        return fminf(1.f, max_norm / (sqrtf(sq) + 1e-6f));
    }
    if (!sqnorm) return 1.f;
    const float total = sqrtf(sqnorm[0]);
    return fminf(1.f, max_norm / (total + 1e-6f));
}

// torch.optim.Adam (_single_tensor_adam, no weight decay / amsgrad):
//   m.lerp_(g, 1-b1); v = v*b2 + (1-b2) g*g; denom = sqrt(v)/bc2_sqrt + eps; p -= step_size*m/denom
__global__ void __launch_bounds__(256) adam_kernel(float *param, const float *grad, float *m, float *v, int64_t n,
                                                   const float *sqnorm, float max_norm, float b1, float b2, float eps,
                                                   float step_size, float bc2_sqrt, SqParts sp) {
    const float coef = clip_coef(sqnorm, sp, max_norm);
    const float w1 = 1.f - b1, w2 = 1.f - b2;
    adam_sweep(param, grad, m, v, n, coef, b2, w1, w2, eps, step_size, bc2_sqrt);
}

// Graph-replay form: the bias corrections from the device-resident step count t and lr (u2gnn_adam_dev),
// formed in double like the host path (torch: lr / (1 - b1^t), sqrt(1 - b2^t)).
__global__ void __launch_bounds__(256) adam_dev_kernel(float *param, const float *grad, float *m, float *v, int64_t n,
                                                       const float *sqnorm, float max_norm, double b1, double b2,
                                                       float eps, const double *lr, const int64_t *t, SqParts sp) {
    const double tt = (double)t[0];
    const float step_size = (float)(lr[0] / (1.0 - pow(b1, tt)));
    const float bc2_sqrt = (float)sqrt(1.0 - pow(b2, tt));
    const float coef = clip_coef(sqnorm, sp, max_norm);
    const float fb1 = (float)b1, fb2 = (float)b2;
    const float w1 = 1.f - fb1, w2 = 1.f - fb2;
    adam_sweep(param, grad, m, v, n, coef, fb2, w1, w2, eps, step_size, bc2_sqrt);
}

__global__ void step_advance_kernel(uint64_t *epoch, int64_t *t) {
    if (epoch) *epoch += 1;
    if (t) *t += 1;
}

// ------------------------------------------------------------------------------------------
// a10 sampled softmax (sampled_softmax.py:36-56).  One block per input row; the sampled
// rows of W are read straight from HBM/L2 (S = 512 rows of D floats, shared by every row).
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) ss_fwd_kernel(const float *X, int64_t ldx, const int64_t *labels,
                                                     const int64_t *sids, int64_t S, const float *W, int64_t ldw,
                                                     float *loss, float *prob, int64_t D) {
    __shared__ float xs[1024];
    __shared__ float red[8];
    const int64_t i = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    // independent loads first: this thread's first two sample ids and the label (the dependent W-row
    // loads follow; the serial chain of the first form cost ~15 us at C5)
    const int64_t sid0 = tid < S ? sids[tid] : 0, sid1 = tid + 256 < S ? sids[tid + 256] : 0;
    const int64_t yl = tid == 0 ? labels[i] : 0;
    for (int64_t c = tid; c < D; c += 256) xs[c] = X[i * ldx + c];
    __syncthreads();
    float tlab = 0.f;
    if (tid == 0) {
        const float *wy = W + yl * ldw;
        for (int64_t c = 0; c < D; ++c) tlab += xs[c] * wy[c];
    }
    float m = -INFINITY, s = 0.f;
    float *pr = prob + i * S;
    for (int64_t j = tid; j < S; j += 256) {
        const float *wr = W + (j == tid ? sid0 : j == tid + 256 ? sid1 : sids[j]) * ldw;
        float dot = 0.f;
        for (int64_t c = 0; c < D; ++c) dot += xs[c] * wr[c];
        pr[j] = dot;  // logits, normalised below
        const float mn = fmaxf(m, dot);
        s = s * expf(m - mn) + expf(dot - mn);
        m = mn;
    }
    const float mw = wave_max(m);
    s = (m == -INFINITY) ? 0.f : s * expf(m - mw);
    s = wave_sum(s);
    if (lane == 0) {
        red[w] = mw;
        red[4 + w] = s;
    }
    __syncthreads();
    const float M = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    float tot = 0.f;
    for (int k = 0; k < 4; ++k) tot += red[k] == -INFINITY ? 0.f : red[4 + k] * expf(red[k] - M);
    const float lse = M + logf(tot);
    for (int64_t j = tid; j < S; j += 256) pr[j] = expf(pr[j] - lse);
    if (tid == 0) loss[i] = lse - tlab;
}

// Block-wide sum of SS_CH per-thread partials (fixed shuffle tree + fixed 4-wave order, so the
// result is deterministic); the totals land in tot[0..SS_CH) for every thread.
constexpr int SS_CH = 8;   // columns per pass (D = d*L is 4 at C5, 19 at C3)
__device__ __forceinline__ void ss_block_sum(float (&acc)[SS_CH], float (*red)[SS_CH], float (&tot)[SS_CH]) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < SS_CH; ++k) acc[k] = wave_sum(acc[k]);
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < SS_CH; ++k) red[w][k] = acc[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < SS_CH; ++k) tot[k] = (red[0][k] + red[1][k]) + (red[2][k] + red[3][k]);
    __syncthreads();
}

// dX[i, c] = g_i (sum_j prob_ij W[s_j, c] - W[y_i, c]); dW[y_i, c] -= g_i X[i, c].
// One block per input row; the S sampled rows are spread over the 256 threads (each thread
// gathers its rows' SS_CH-column slices: independent loads, no serial latency chain over S).
// ROWS (ABI v9): the label term is stored as compact row i of dW (ld lddw) instead of added at y_i.
template <bool ROWS>
__global__ void __launch_bounds__(256) ss_bwd_x_kernel(const float *X, int64_t ldx, const int64_t *labels,
                                                       const int64_t *sids, int64_t S, const float *W, int64_t ldw,
                                                       const float *prob, const float *dloss, float *dX, int64_t lddx,
                                                       float *dW, int64_t lddw, int64_t D) {
    __shared__ float red[4][SS_CH];
    const int64_t i = blockIdx.x;
    const int tid = threadIdx.x;
    const float g = dloss ? dloss[i] : 1.f;
    const float *pr = prob + i * S;
    const int64_t y = labels[i];
    for (int64_t c0 = 0; c0 < D; c0 += SS_CH) {
        float acc[SS_CH], tot[SS_CH];
#pragma unroll
        for (int k = 0; k < SS_CH; ++k) acc[k] = 0.f;
        int64_t j0 = tid;
        for (; j0 + 256 < S; j0 += 512) {   // two samples' loads in flight, summed in sample order
            const float p0 = pr[j0], p1 = pr[j0 + 256];
            const float *w0 = W + sids[j0] * ldw + c0, *w1 = W + sids[j0 + 256] * ldw + c0;
            float v0[SS_CH], v1[SS_CH];
#pragma unroll
            for (int k = 0; k < SS_CH; ++k) {
                v0[k] = c0 + k < D ? w0[k] : 0.f;
                v1[k] = c0 + k < D ? w1[k] : 0.f;
            }
#pragma unroll
            for (int k = 0; k < SS_CH; ++k)
                if (c0 + k < D) acc[k] += p0 * v0[k];
#pragma unroll
            for (int k = 0; k < SS_CH; ++k)
                if (c0 + k < D) acc[k] += p1 * v1[k];
        }
        for (int64_t j = j0; j < S; j += 256) {
            const float pj = pr[j];
            const float *wr = W + sids[j] * ldw + c0;
#pragma unroll
            for (int k = 0; k < SS_CH; ++k)
                if (c0 + k < D) acc[k] += pj * wr[k];
        }
        ss_block_sum(acc, red, tot);
        if (tid < SS_CH && c0 + tid < D) {
            float t = tot[0];
#pragma unroll
            for (int k = 1; k < SS_CH; ++k)
                if (tid == k) t = tot[k];
            const int64_t c = c0 + tid;
            dX[i * lddx + c] = g * (t - W[y * ldw + c]);
            if constexpr (ROWS)
                dW[i * lddw + c] = -g * X[i * ldx + c];
            else
                atomicAdd(dW + y * lddw + c, -g * X[i * ldx + c]);
        }
    }
}

// dW[s_j, c] += sum_i g_i prob_ij X[i, c]; one block per sample j, the input rows spread over
// the 256 threads (independent loads), deterministic block sum.  ROWS: stored as compact row j.
template <bool ROWS>
__global__ void __launch_bounds__(256) ss_bwd_w_kernel(const float *X, int64_t ldx, const int64_t *sids, int64_t S,
                                                       const float *prob, const float *dloss, float *dW, int64_t lddw,
                                                       int64_t n_rows, int64_t D) {
    __shared__ float red[4][SS_CH];
    const int64_t j = blockIdx.x;
    const int tid = threadIdx.x;
    float *dw = dW + (ROWS ? j : sids[j]) * lddw;
    for (int64_t c0 = 0; c0 < D; c0 += SS_CH) {
        float acc[SS_CH], tot[SS_CH];
#pragma unroll
        for (int k = 0; k < SS_CH; ++k) acc[k] = 0.f;
        // 8 rows' loads in flight per thread (the strided prob column and the X rows), then the FMAs in
        // row order (the same sums as one row at a time)
        int64_t i0 = tid;
        for (; i0 + 7 * 256 < n_rows; i0 += 8 * 256) {
            float f[8], xv[8][SS_CH];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int64_t i = i0 + u * 256;
                f[u] = (dloss ? dloss[i] : 1.f) * prob[i * S + j];
#pragma unroll
                for (int k = 0; k < SS_CH; ++k) xv[u][k] = c0 + k < D ? X[i * ldx + c0 + k] : 0.f;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u)
#pragma unroll
                for (int k = 0; k < SS_CH; ++k)
                    if (c0 + k < D) acc[k] += f[u] * xv[u][k];
        }
        for (int64_t i = i0; i < n_rows; i += 256) {
            const float f = (dloss ? dloss[i] : 1.f) * prob[i * S + j];
            const float *xr = X + i * ldx + c0;
#pragma unroll
            for (int k = 0; k < SS_CH; ++k)
                if (c0 + k < D) acc[k] += f * xr[k];
        }
        ss_block_sum(acc, red, tot);
        if (tid < SS_CH && c0 + tid < D) {
            float t = tot[0];
#pragma unroll
            for (int k = 1; k < SS_CH; ++k)
                if (tid == k) t = tot[k];
            if constexpr (ROWS)
                dw[c0 + tid] = t;
            else
                atomicAdd(dw + c0 + tid, t);
        }
    }
}

// dst[idx[r], c] (+)= alpha * src[r, c]: one wave per row, the row's columns over the lanes.  ZERO:
// dst[idx[r], c] = 0 (src unused).  Destinations of one launch are distinct (u2gnn_hip.h), so the
// read-modify-write needs no atomics.
template <bool ZERO>
__global__ void __launch_bounds__(256) index_rows_kernel(const float *src, int64_t ld_src, const int64_t *idx,
                                                         int64_t n_rows, float alpha, float *dst, int64_t ld_dst,
                                                         int64_t dst_rows, int64_t D, int32_t *err) {
    const int lane = threadIdx.x & 63;
    for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < n_rows; r += (int64_t)gridDim.x * 4) {
        const int64_t y = idx[r];
        if (y < 0 || y >= dst_rows) {
            if (err && lane == 0) *err = 1;
            continue;
        }
        float *d = dst + y * ld_dst;
        for (int64_t c = lane; c < D; c += 64) {
            if constexpr (ZERO)
                d[c] = 0.f;
            else
                d[c] += alpha * src[r * ld_src + c];
        }
    }
}

inline unsigned grid_for(int64_t n, int64_t per_block, int64_t cap = 8192) {
    int64_t g = (n + per_block - 1) / per_block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}

// ------------------------------------------------------------------------------------------
// UnSup head glue (ABI v11; pytorch_U2GNN_UnSup.py:52-69 + the TF model's dropout before the sampled
// softmax, U2GNN_tf/model_U2GNN_Unsup_multi.py:43-56).  concat_dropout: the L layers' padded slot-0
// outputs -> Y[N, d*L] with dropout(p) (the mask of u2gnn_dropout over Y's (row, column) indices) in one
// pass; split_dropout_bwd: the gradient of that, dropped out with the same mask and written back as
// L zero-padded [Np][dp] images (u2gnn_dropout + L u2gnn_pack_padded in one pass).
// ------------------------------------------------------------------------------------------
constexpr int CAT_MAX = 8;
struct CatSrc {
    const float *p[CAT_MAX];
};
struct CatDst {
    float *p[CAT_MAX];
};

__global__ void __launch_bounds__(256) concat_dropout_kernel(CatSrc src, int64_t ld_src, int64_t N, int64_t d, int L,
                                                             float p, uint64_t seed, const uint64_t *seed_epoch,
                                                             float *Y, int64_t ldy) {
    seed = u2gnn_seed(seed, seed_epoch);
    const int64_t D = d * L, total = N * D;
    const float ks = 1.f / (1.f - p);
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        const int64_t r = i / D, c = i - r * D, l = c / d;
        const float v = src.p[l][r * ld_src + (c - l * d)];
        Y[r * ldy + c] = p > 0.f ? (u2gnn_keep(seed, (uint32_t)r, (uint32_t)c, p) ? v * ks : 0.f) : v;
    }
}

__global__ void __launch_bounds__(256) split_dropout_bwd_kernel(const float *dY, int64_t ldy, int64_t N, int64_t Np,
                                                                int64_t d, int64_t dp, int L, float p, uint64_t seed,
                                                                const uint64_t *seed_epoch, CatDst dst) {
    seed = u2gnn_seed(seed, seed_epoch);
    const int64_t per = Np * dp, total = per * L;
    const float ks = 1.f / (1.f - p);
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        const int64_t l = i / per, e = i - l * per, r = e / dp, c = e - r * dp;
        float v = 0.f;
        if (r < N && c < d) {
            const int64_t cc = l * d + c;
            v = dY[r * ldy + cc];
            if (p > 0.f) v = u2gnn_keep(seed, (uint32_t)r, (uint32_t)cc, p) ? v * ks : 0.f;
        }
        dst.p[l][e] = v;
    }
}

// out[0] = sum of x[0, n): one 1024-thread block, lane t sums x[t], x[t + 1024], ... (4 accumulators), then
// a fixed shuffle / LDS tree (deterministic)
__global__ void __launch_bounds__(1024) sum_kernel(const float *x, int64_t n, float *out) {
    __shared__ float red[16];
    float a[4] = {0.f, 0.f, 0.f, 0.f};
    int64_t i = threadIdx.x;
    for (; i + 3 * 1024 < n; i += 4 * 1024) {
#pragma unroll
        for (int k = 0; k < 4; ++k) a[k] += x[i + k * 1024];
    }
    for (; i < n; i += 1024) a[0] += x[i];
    float s = wave_sum((a[0] + a[1]) + (a[2] + a[3]));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        float t = 0.f;
        for (int w = 0; w < 16; ++w) t += red[w];
        out[0] = t;
    }
}

// dst[idx_a[r]] = 0 and dst[idx_b[r]] = 0 in one launch (zeroing is idempotent: the sets may overlap)
__global__ void __launch_bounds__(256) index_zero_rows2_kernel(const int64_t *ia, int64_t na, const int64_t *ib,
                                                               int64_t nb, float *dst, int64_t ld_dst, int64_t dst_rows,
                                                               int64_t D, int32_t *err) {
    const int lane = threadIdx.x & 63;
    for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < na + nb; r += (int64_t)gridDim.x * 4) {
        const int64_t y = r < na ? ia[r] : ib[r - na];
        if (y < 0 || y >= dst_rows) {
            if (err && lane == 0) *err = 1;
            continue;
        }
        for (int64_t c = lane; c < D; c += 64) dst[y * ld_dst + c] = 0.f;
    }
}

}  // namespace

extern "C" {

int u2gnn_concat_dropout(const float *const *src, int32_t L, int64_t ld_src, int64_t N, int64_t d, float p,
                         uint64_t seed, float *Y, int64_t ldy, void *stream) {
    if (!src || L < 1 || L > CAT_MAX || N < 0 || d < 1 || ld_src < d || !Y || ldy < d * L || p < 0.f || p >= 1.f)
        return U2GNN_E_ARG;
    CatSrc cs;
    for (int l = 0; l < CAT_MAX; ++l) cs.p[l] = l < L ? src[l] : nullptr;
    for (int l = 0; l < L; ++l)
        if (!cs.p[l]) return U2GNN_E_ARG;
    if (N == 0) return U2GNN_OK;
    hipLaunchKernelGGL(concat_dropout_kernel, dim3(grid_for(N * d * L, 256)), dim3(256), 0, u2gnn_stream(stream), cs,
                       ld_src, N, d, (int)L, p, seed, u2gnn_cur_epoch(), Y, ldy);
    return u2gnn_launch_status();
}

int u2gnn_split_dropout_bwd(const float *dY, int64_t ldy, int32_t L, int64_t N, int64_t Np, int64_t d, int64_t dp,
                            float p, uint64_t seed, float *const *dst, void *stream) {
    if (!dY || !dst || L < 1 || L > CAT_MAX || N < 0 || Np < N || d < 1 || dp < d || ldy < d * L || p < 0.f ||
        p >= 1.f)
        return U2GNN_E_ARG;
    CatDst cd;
    for (int l = 0; l < CAT_MAX; ++l) cd.p[l] = l < L ? dst[l] : nullptr;
    for (int l = 0; l < L; ++l)
        if (!cd.p[l]) return U2GNN_E_ARG;
    if (Np == 0) return U2GNN_OK;
    hipLaunchKernelGGL(split_dropout_bwd_kernel, dim3(grid_for(Np * dp * L, 256)), dim3(256), 0, u2gnn_stream(stream),
                       dY, ldy, N, Np, d, dp, (int)L, p, seed, u2gnn_cur_epoch(), cd);
    return u2gnn_launch_status();
}

int u2gnn_sum(const float *x, int64_t n, float *out, void *stream) {
    if (!x || !out || n < 0) return U2GNN_E_ARG;
    hipLaunchKernelGGL(sum_kernel, dim3(1), dim3(1024), 0, u2gnn_stream(stream), x, n, out);
    return u2gnn_launch_status();
}

int u2gnn_index_zero_rows2(const int64_t *idx_a, int64_t n_a, const int64_t *idx_b, int64_t n_b, float *dst,
                           int64_t ld_dst, int64_t dst_rows, int64_t D, int32_t *err, void *stream) {
    if (n_a < 0 || n_b < 0 || D < 0) return U2GNN_E_ARG;
    if (n_a + n_b == 0 || D == 0) return U2GNN_OK;
    if ((n_a && !idx_a) || (n_b && !idx_b) || !dst || ld_dst < D) return U2GNN_E_ARG;
    hipLaunchKernelGGL(index_zero_rows2_kernel, dim3(grid_for(n_a + n_b, 4, 1 << 20)), dim3(256), 0,
                       u2gnn_stream(stream), idx_a, n_a, idx_b, n_b, dst, ld_dst, dst_rows, D, err);
    return u2gnn_launch_status();
}

int u2gnn_pool_fwd(const float *X, int64_t ldx, const int64_t *rowptr, const int64_t *colidx, const float *vals,
                   float *G, int64_t ldg, int64_t B, int64_t d, float p, uint64_t seed, void *stream) {
    if (!X || !rowptr || !colidx || !vals || !G || B < 1 || d < 1) return U2GNN_E_ARG;
    hipLaunchKernelGGL(pool_fwd_kernel, dim3((unsigned)B, (unsigned)((d + 63) / 64)), dim3(64 * POOL_WAVES), 0,
                       u2gnn_stream(stream), X, ldx, rowptr, colidx, vals, G, ldg, d, p, seed, u2gnn_cur_epoch());
    return u2gnn_launch_status();
}

int u2gnn_pool_bwd(const float *dGd, int64_t ldg, const int64_t *rowptr, const int64_t *colidx, const float *vals,
                   float *dX, int64_t ldx, int64_t B, int64_t d, float p, uint64_t seed, void *stream) {
    if (!dGd || !rowptr || !colidx || !vals || !dX || B < 1 || d < 1) return U2GNN_E_ARG;
    hipLaunchKernelGGL(pool_bwd_kernel, dim3((unsigned)B, 8, (unsigned)((d + 63) / 64)), dim3(256), 0,
                       u2gnn_stream(stream), dGd, ldg, rowptr, colidx, vals, dX, ldx, d, p, seed, u2gnn_cur_epoch());
    return u2gnn_launch_status();
}

int u2gnn_pool_bwd_rows(const float *dGd, int64_t ldg, const int64_t *rowptr, const int64_t *colidx,
                        const float *vals, float *dX, int64_t ldx, int64_t B, int64_t d, int64_t d_pad, int64_t N,
                        int64_t rows_pad, float p, uint64_t seed, void *stream) {
    if (!dGd || !rowptr || !colidx || !vals || !dX || B < 1 || d < 1 || d > d_pad || d_pad > ldx || N < 0 ||
        N > rows_pad)
        return U2GNN_E_ARG;
    const int64_t zb = (rows_pad - N + 31) / 32;   // padding-row blocks: 8 x 4 waves, one row each
    hipLaunchKernelGGL(pool_bwd_rows_kernel, dim3((unsigned)(B + zb), 8, (unsigned)((d_pad + 63) / 64)), dim3(256), 0,
                       u2gnn_stream(stream), dGd, ldg, rowptr, colidx, vals, dX, ldx, B, d, d_pad, N, rows_pad, p,
                       seed, u2gnn_cur_epoch());
    return u2gnn_launch_status();
}

int u2gnn_head_fwd(const float *G, int64_t ldg, const float *W, const float *bias, float *scores, int64_t B, int64_t C,
                   int64_t d, int32_t accumulate, void *stream) {
    if (!G || !W || !bias || !scores || B < 1 || C < 1) return U2GNN_E_ARG;
    hipLaunchKernelGGL(head_fwd_kernel, dim3(grid_for(B * C, 4, 1 << 30)), dim3(256), 0, u2gnn_stream(stream), G, ldg,
                       W, bias, scores, B, C, d, accumulate);
    return u2gnn_launch_status();
}

int u2gnn_head_bwd(const float *dscores, const float *G, int64_t ldg, const float *W, float *dG, int64_t lddg,
                   float *dW, float *db, int64_t B, int64_t C, int64_t d, int32_t accumulate, void *stream) {
    if (!dscores || !G || !W || !dG || !dW || !db) return U2GNN_E_ARG;
    hipLaunchKernelGGL(head_bwd_kernel, dim3(grid_for(B * d + C * d + C, 256, 1 << 30)), dim3(256), 0, u2gnn_stream(stream), dscores,
                       G, ldg, W, dG, lddg, dW, db, B, C, d, accumulate);
    return u2gnn_launch_status();
}

int u2gnn_smoothed_ce(const float *scores, const int64_t *labels, int64_t B, int64_t C, float smoothing, float *loss,
                      float *dscores, void *stream) {
    if (!scores || !labels || !loss || !dscores || B < 1 || C < 2) return U2GNN_E_ARG;
    hipLaunchKernelGGL(smoothed_ce_kernel, dim3(1), dim3(256), 0, u2gnn_stream(stream), scores, labels, B, C,
                       smoothing, loss, dscores);
    return u2gnn_launch_status();
}

namespace {
inline unsigned sqnorm_blocks(int64_t n) { return grid_for(n, 256 * 16, 512); }   // ws holds 512 doubles
}  // namespace

int u2gnn_sqnorm_partials(const float *g, int64_t n, float *ws, void *stream) {
    if (!g || !ws || (reinterpret_cast<uintptr_t>(g) & 15)) return U2GNN_E_ARG;
    hipLaunchKernelGGL(sqnorm_partial_kernel, dim3(sqnorm_blocks(n)), dim3(256), 0, u2gnn_stream(stream), g, n,
                       reinterpret_cast<double *>(ws));
    return u2gnn_launch_status();
}

int u2gnn_adam_sq(float *param, const float *grad, float *exp_avg, float *exp_avg_sq, int64_t n, const float *ws,
                  float *sqnorm, float max_norm, float beta1, float beta2, float eps, float step_size, float bc2_sqrt,
                  void *stream) {
    if (!param || !grad || !exp_avg || !exp_avg_sq || !ws) return U2GNN_E_ARG;
    if (n == 0) return U2GNN_OK;
    const SqParts sp{reinterpret_cast<const double *>(ws), (int)sqnorm_blocks(n), sqnorm};
    hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n, 1024, 4096)), dim3(256), 0, u2gnn_stream(stream), param, grad,
                       exp_avg, exp_avg_sq, n, nullptr, max_norm, beta1, beta2, eps, step_size, bc2_sqrt, sp);
    return u2gnn_launch_status();
}

int u2gnn_adam_dev_sq(float *param, const float *grad, float *exp_avg, float *exp_avg_sq, int64_t n, const float *ws,
                      float *sqnorm, float max_norm, double beta1, double beta2, float eps, const double *lr,
                      const int64_t *step, void *stream) {
    if (!param || !grad || !exp_avg || !exp_avg_sq || !ws || !lr || !step) return U2GNN_E_ARG;
    if (n == 0) return U2GNN_OK;
    const SqParts sp{reinterpret_cast<const double *>(ws), (int)sqnorm_blocks(n), sqnorm};
    hipLaunchKernelGGL(adam_dev_kernel, dim3(grid_for(n, 1024, 4096)), dim3(256), 0, u2gnn_stream(stream), param, grad,
                       exp_avg, exp_avg_sq, n, nullptr, max_norm, beta1, beta2, eps, lr, step, sp);
    return u2gnn_launch_status();
}

int u2gnn_sqnorm(const float *g, int64_t n, float *ws, float *sqnorm, void *stream) {
    if (!g || !ws || !sqnorm || (reinterpret_cast<uintptr_t>(g) & 15)) return U2GNN_E_ARG;
    const unsigned nb = sqnorm_blocks(n);
    hipStream_t st = u2gnn_stream(stream);
    double *wsd = reinterpret_cast<double *>(ws);
    hipLaunchKernelGGL(sqnorm_partial_kernel, dim3(nb), dim3(256), 0, st, g, n, wsd);
    hipLaunchKernelGGL(sqnorm_final_kernel, dim3(1), dim3(256), 0, st, wsd, (int)nb, sqnorm);
    return u2gnn_launch_status();
}

int u2gnn_adam(float *param, const float *grad, float *exp_avg, float *exp_avg_sq, int64_t n, const float *sqnorm,
               float max_norm, float beta1, float beta2, float eps, float step_size, float bc2_sqrt, void *stream) {
    if (!param || !grad || !exp_avg || !exp_avg_sq) return U2GNN_E_ARG;
    if (n == 0) return U2GNN_OK;
    hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n, 1024, 4096)), dim3(256), 0, u2gnn_stream(stream), param, grad,
                       exp_avg, exp_avg_sq, n, sqnorm, max_norm, beta1, beta2, eps, step_size, bc2_sqrt,
                       SqParts{nullptr, 0, nullptr});
    return u2gnn_launch_status();
}

int u2gnn_adam_dev(float *param, const float *grad, float *exp_avg, float *exp_avg_sq, int64_t n, const float *sqnorm,
                   float max_norm, double beta1, double beta2, float eps, const double *lr, const int64_t *step,
                   void *stream) {
    if (!param || !grad || !exp_avg || !exp_avg_sq || !lr || !step) return U2GNN_E_ARG;
    if (n == 0) return U2GNN_OK;
    hipLaunchKernelGGL(adam_dev_kernel, dim3(grid_for(n, 1024, 4096)), dim3(256), 0, u2gnn_stream(stream), param, grad,
                       exp_avg, exp_avg_sq, n, sqnorm, max_norm, beta1, beta2, eps, lr, step,
                       SqParts{nullptr, 0, nullptr});
    return u2gnn_launch_status();
}

int u2gnn_step_advance(uint64_t *epoch, int64_t *step, void *stream) {
    if (!epoch && !step) return U2GNN_OK;
    hipLaunchKernelGGL(step_advance_kernel, dim3(1), dim3(1), 0, u2gnn_stream(stream), epoch, step);
    return u2gnn_launch_status();
}

int u2gnn_set_seed_epoch(const uint64_t *epoch) {
    const int d = current_device();
    if (d < 0) return U2GNN_E_ARG;
    g_epoch[d].store(epoch, std::memory_order_release);
    return U2GNN_OK;
}

int u2gnn_sampled_softmax_fwd(const float *X, int64_t ldx, const int64_t *labels, const int64_t *sample_ids, int64_t S,
                              const float *W, int64_t ldw, float *loss, float *prob, int64_t n_rows, int64_t D,
                              void *stream) {
    if (!X || !labels || !sample_ids || !W || !loss || !prob || D > 1024 || S < 1) return U2GNN_E_ARG;
    if (n_rows == 0) return U2GNN_OK;
    hipLaunchKernelGGL(ss_fwd_kernel, dim3((unsigned)n_rows), dim3(256), 0, u2gnn_stream(stream), X, ldx, labels,
                       sample_ids, S, W, ldw, loss, prob, D);
    return u2gnn_launch_status();
}

int u2gnn_sampled_softmax_bwd(const float *X, int64_t ldx, const int64_t *labels, const int64_t *sample_ids, int64_t S,
                              const float *W, int64_t ldw, const float *prob, const float *dloss, float *dX,
                              int64_t lddx, float *dW, int64_t lddw, int64_t n_rows, int64_t D, void *stream) {
    if (!X || !labels || !sample_ids || !W || !prob || !dX || !dW || S < 1) return U2GNN_E_ARG;
    if (n_rows == 0) return U2GNN_OK;
    hipStream_t st = u2gnn_stream(stream);
    hipLaunchKernelGGL(ss_bwd_x_kernel<false>, dim3((unsigned)n_rows), dim3(256), 0, st, X, ldx, labels, sample_ids, S,
                       W, ldw, prob, dloss, dX, lddx, dW, lddw, D);
    hipLaunchKernelGGL(ss_bwd_w_kernel<false>, dim3((unsigned)S), dim3(256), 0, st, X, ldx, sample_ids, S, prob, dloss,
                       dW, lddw, n_rows, D);
    return u2gnn_launch_status();
}

int u2gnn_sampled_softmax_bwd_rows(const float *X, int64_t ldx, const int64_t *labels, const int64_t *sample_ids,
                                   int64_t S, const float *W, int64_t ldw, const float *prob, const float *dloss,
                                   float *dX, int64_t lddx, float *dW_lab, int64_t ld_lab, float *dW_smp,
                                   int64_t ld_smp, int64_t n_rows, int64_t D, void *stream) {
    if (!X || !labels || !sample_ids || !W || !prob || !dX || !dW_smp || S < 1 || D < 1) return U2GNN_E_ARG;
    if (n_rows > 0 && !dW_lab) return U2GNN_E_ARG;
    if (ld_lab < D || ld_smp < D) return U2GNN_E_ARG;
    hipStream_t st = u2gnn_stream(stream);
    if (n_rows > 0)
        hipLaunchKernelGGL(ss_bwd_x_kernel<true>, dim3((unsigned)n_rows), dim3(256), 0, st, X, ldx, labels, sample_ids,
                           S, W, ldw, prob, dloss, dX, lddx, dW_lab, ld_lab, D);
    hipLaunchKernelGGL(ss_bwd_w_kernel<true>, dim3((unsigned)S), dim3(256), 0, st, X, ldx, sample_ids, S, prob, dloss,
                       dW_smp, ld_smp, n_rows, D);
    return u2gnn_launch_status();
}

int u2gnn_index_add_rows(const float *src, int64_t ld_src, const int64_t *idx, int64_t n_rows, float alpha,
                         float *dst, int64_t ld_dst, int64_t dst_rows, int64_t D, int32_t *err, void *stream) {
    if (n_rows < 0 || D < 0) return U2GNN_E_ARG;
    if (n_rows == 0 || D == 0) return U2GNN_OK;
    if (!src || !idx || !dst || ld_src < D || ld_dst < D) return U2GNN_E_ARG;
    hipLaunchKernelGGL(index_rows_kernel<false>, dim3(grid_for(n_rows, 4, 1 << 20)), dim3(256), 0,
                       u2gnn_stream(stream), src, ld_src, idx, n_rows, alpha, dst, ld_dst, dst_rows, D, err);
    return u2gnn_launch_status();
}

int u2gnn_index_zero_rows(const int64_t *idx, int64_t n_rows, float *dst, int64_t ld_dst, int64_t dst_rows, int64_t D,
                          int32_t *err, void *stream) {
    if (n_rows < 0 || D < 0) return U2GNN_E_ARG;
    if (n_rows == 0 || D == 0) return U2GNN_OK;
    if (!idx || !dst || ld_dst < D) return U2GNN_E_ARG;
    hipLaunchKernelGGL(index_rows_kernel<true>, dim3(grid_for(n_rows, 4, 1 << 20)), dim3(256), 0,
                       u2gnn_stream(stream), nullptr, 0, idx, n_rows, 0.f, dst, ld_dst, dst_rows, D, err);
    return u2gnn_launch_status();
}

int u2gnn_abi_version(void) { return U2GNN_ABI_VERSION; }

}  // extern "C"
