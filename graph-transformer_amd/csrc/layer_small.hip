// Row-local tail of a small-width encoder layer (d <= 32: the UnSup encoders REDDIT-M5K d = 4 (C5), PTC
// d = 19 (C3), MUTAG d = 7) -- a3.3 + a3.4 of SURVEY.md §8 and their backward, one launch each way
// (torch.nn.TransformerEncoderLayer inside pytorch_U2GNN_UnSup.py:37-40,57 / pytorch_U2GNN_Sup.py:19-21,35:
// out_proj -> dropout1 -> + x -> norm1 -> linear1 -> ReLU -> dropout -> linear2 -> dropout2 -> + x -> norm2).
//
// Everything after the attention is row-local: with d <= 32 a row is d values and its FFN is 2 ff d
// multiply-adds, so the matrix-core form (dp = 64 padded GEMMs with 94 % padding at d = 4, plus split-K slabs and
// LayerNorm passes: 3-5 launches of a few microseconds each way, latency-bound) gives way to one wave per row
// in exact fp32 on the vector ALUs:
//   forward   lane c < d: z1 = drop1(O W_o^T + b_o) + x, LayerNorm1 -> x1 (wave sums); then the lanes split
//             the ff hidden units (LDS-staged chunks of W1 and W2^T, compact d-wide rows): h = dropff(relu(x1
//             W1^T + b1)) written to Hd, the d partial sums of h W2^T reduced over the wave; lane c: z2 =
//             drop2(. + b2) + x1, LayerNorm2 -> x2.
//   backward  LayerNorm2^T -> dF = drop2'(dz2); the lanes split the hidden units again: dH = (Hd > 0) dF W2 /
//             (1-p), dX1 = dz2 + dH W1 (wave sums); LayerNorm1^T -> dX (residual) and dA = drop1'(dz1); dO =
//             dA W_o and delta = rowsum(dO * O) for the attention backward.
// The parameter gradients (column sums over the rows) stay with the executor's side-stream reductions, which
// read dF, dH, dA, dX1 as written here.  Dropout: u2gnn_keep(seed, row, column) of every site, the same bits as
// the GEMM epilogues'.  Deterministic: fixed hidden-unit partition and butterfly sums.
#include <cmath>
#include <cstring>

#include "u2gnn_common.h"

namespace {

constexpr int LS_WAVES = 8;                // rows per 512-thread workgroup (one wave per row)
constexpr int LS_NT = 64 * LS_WAVES;
// hidden units per LDS chunk: W1 and W2^T chunks of HC x DM floats each (32 KB together)
template <int DM> constexpr int ls_hc() { return 4096 / DM / 64 * 64; }
template <int DM> constexpr int ls_min_waves() { return DM <= 16 ? 4 : 2; }

struct LsP {
    int32_t N, Np, d, dp, ff, ffp;
    float p, eps;
    uint64_t s1, sff, s2;
    const uint64_t *epoch;
    u2gnn_small_tail_args a;
};

__device__ __forceinline__ float wsum(float v) { return wave_sum(v); }

// v (the same in every lane) -> lane c gets v[c] (0 past DM)
template <int DM>
__device__ __forceinline__ float pick(const float (&v)[DM], int c) {
    float r = 0.f;
#pragma unroll
    for (int k = 0; k < DM; ++k) r = c == k ? v[k] : r;
    return r;
}

// Staging of hidden units [h0, h0 + HC): W1 [ffp][dp] (rows, first DM columns), W2 [dp][ffp] (first DM rows,
// transposed: w2s[h][c] = W2[c][h]) and, for the forward, b1 into LDS; units at or past ffp are zeros.  load()
// issues every global load of the chunk into registers (all in flight together), store() writes them to LDS:
// one load latency per chunk instead of one per loop iteration (a load -> ds_write loop waits on every load).
template <int DM, int HC, bool BIAS>
struct Stage {
    static constexpr int C4 = DM / 4, N1 = HC * C4, N2 = DM * (HC / 4), N3 = BIAS ? HC / 4 : 0;
    static constexpr int P1 = (N1 + LS_NT - 1) / LS_NT, P2 = (N2 + LS_NT - 1) / LS_NT, P3 = (N3 + LS_NT - 1) / LS_NT;
    float4 a[P1], b[P2], c[P3 > 0 ? P3 : 1];
    __device__ __forceinline__ void load(const LsP &P, int h0) {
        const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int i = 0; i < P1; ++i) {
            const int e = threadIdx.x + i * LS_NT, h = e / C4, k = 4 * (e % C4);
            a[i] = z;
            if (e < N1 && h0 + h < P.ffp) a[i] = *reinterpret_cast<const float4 *>(P.a.W1 + (int64_t)(h0 + h) * P.dp + k);
        }
#pragma unroll
        for (int i = 0; i < P2; ++i) {   // W2 row k, 4 consecutive hidden units: coalesced
            const int e = threadIdx.x + i * LS_NT, k = e / (HC / 4), h = 4 * (e % (HC / 4));
            b[i] = z;
            if (e < N2 && h0 + h < P.ffp) b[i] = *reinterpret_cast<const float4 *>(P.a.W2 + (int64_t)k * P.ffp + h0 + h);
        }
#pragma unroll
        for (int i = 0; i < P3; ++i) {
            const int e = threadIdx.x + i * LS_NT, h = 4 * e;
            c[i] = z;
            if (e < N3 && h0 + h < P.ffp) c[i] = *reinterpret_cast<const float4 *>(P.a.b1 + h0 + h);
        }
    }
    __device__ __forceinline__ void store(float (*w1s)[DM], float (*w2s)[DM], float *b1s) const {
#pragma unroll
        for (int i = 0; i < P1; ++i) {
            const int e = threadIdx.x + i * LS_NT;
            if (e < N1) *reinterpret_cast<float4 *>(&w1s[e / C4][4 * (e % C4)]) = a[i];
        }
#pragma unroll
        for (int i = 0; i < P2; ++i) {
            const int e = threadIdx.x + i * LS_NT, k = e / (HC / 4), h = 4 * (e % (HC / 4));
            if (e < N2) w2s[h][k] = b[i].x, w2s[h + 1][k] = b[i].y, w2s[h + 2][k] = b[i].z, w2s[h + 3][k] = b[i].w;
        }
#pragma unroll
        for (int i = 0; i < P3; ++i) {
            const int e = threadIdx.x + i * LS_NT;
            if (e < N3) *reinterpret_cast<float4 *>(b1s + 4 * e) = c[i];
        }
    }
};

// post-LN of one row held as lane c < d: returns y_c (0 past d), the row's mean and 1/std
__device__ __forceinline__ float ln_row(float z, int lane, int d, float eps, const float *gamma, const float *beta,
                                        float &mu, float &rs) {
    const bool ok = lane < d;
    const float v = ok ? z : 0.f;
    mu = wsum(v) / (float)d;
    const float t = ok ? v - mu : 0.f;
    rs = rsqrtf(wsum(t * t) / (float)d + eps);
    const int c = ok ? lane : 0;   // gamma, beta: unpadded [d]
    return ok ? t * rs * gamma[c] + beta[c] : 0.f;
}

// LN backward of one row (lane c < d): dz = rs (g - mean(g) - xh mean(g xh)), g = dy gamma, xh = (z - mu) rs
__device__ __forceinline__ float ln_row_bwd(float dy, float z, float mu, float rs, int lane, int d, const float *gamma) {
    const bool ok = lane < d;
    const float xh = ok ? (z - mu) * rs : 0.f;
    const float g = ok ? dy * gamma[ok ? lane : 0] : 0.f;
    const float m1 = wsum(g) / (float)d, m2 = wsum(g * xh) / (float)d;
    return ok ? rs * (g - m1 - xh * m2) : 0.f;
}

// Two work splits.  STAGED (large N, e.g. C5's 2048 rows): 8 rows per workgroup, one wave per row, the weights
// staged through LDS in chunks of HC hidden units and shared by the 8 rows.  DIRECT (N < 1024 padded rows, e.g.
// C3's 128: the staged split leaves most CUs idle): one row per workgroup, its 8 waves splitting the hidden units
// (unit 64 (w + 8 u) + lane), each wave's W1 / W2 / b1 values loaded straight from L2 into registers (no LDS
// staging, no chunk barriers), the 8 waves' partial sums combined through LDS in wave order.
template <bool DIRECT> __device__ __forceinline__ int ls_row() {
    return DIRECT ? (int)blockIdx.x : (int)blockIdx.x * LS_WAVES + (int)(threadIdx.x >> 6);
}

// one hidden unit of the forward: h = dropff(relu(b1 + x1 . W1[h])), written to Hd; zp += h W2[:, h]
template <int DM>
__device__ __forceinline__ void ffn_unit_fwd(const float (&xv)[DM], const float (&w1)[DM], const float (&w2)[DM], float b,
                                             bool keep, float ks, bool live, float *dst, float (&zp)[DM]) {
    float a = b;
#pragma unroll
    for (int k = 0; k < DM; ++k) a = fmaf(xv[k], w1[k], a);
    a = fmaxf(a, 0.f);
    a = keep ? a * ks : 0.f;
    if (!live) a = 0.f;
    *dst = a;
#pragma unroll
    for (int k = 0; k < DM; ++k) zp[k] = fmaf(a, w2[k], zp[k]);
}

template <int DM, bool DIRECT>
__global__ void __launch_bounds__(LS_NT, ls_min_waves<DM>()) ls_fwd_kernel(LsP P) {
    constexpr int HC = DIRECT ? 64 : ls_hc<DM>(), NU = HC / 64;
    __shared__ __attribute__((aligned(16))) float w1s[DIRECT ? 1 : HC][DM];
    __shared__ __attribute__((aligned(16))) float w2s[DIRECT ? 1 : HC][DM];
    __shared__ float b1s[DIRECT ? 1 : HC];
    __shared__ float xw[DIRECT ? LS_WAVES : 1][DM];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r = ls_row<DIRECT>();   // < Np (Np % 8 == 0, host-checked)
    const bool live = r < P.N;
    const bool writer = !DIRECT || w == 0;   // DIRECT: every wave computes the row prologue, wave 0 stores it
    const u2gnn_small_tail_args &A = P.a;
    const bool drop = P.p > 0.f;
    const float ks = drop ? 1.f / (1.f - P.p) : 1.f;
    const uint32_t thr = u2gnn_keep_thr(P.p);
    const uint64_t s1 = u2gnn_seed(P.s1, P.epoch), sff = u2gnn_seed(P.sff, P.epoch), s2 = u2gnn_seed(P.s2, P.epoch);
    const int64_t ro = (int64_t)r * P.dp;
    // a3.3: z1 = drop1(O W_o^T + b_o) + x (lane c), LayerNorm1
    float x1 = 0.f, mu1 = 0.f, rs1 = 0.f, z1 = 0.f;
    float xv[DM];
#pragma unroll
    for (int k = 0; k < DM; ++k) xv[k] = 0.f;
    if (live) {
        float o[DM], wo[DM];
#pragma unroll
        for (int k = 0; k < DM; k += 4) {
            const float4 t = *reinterpret_cast<const float4 *>(A.O + ro + k);
            o[k] = t.x, o[k + 1] = t.y, o[k + 2] = t.z, o[k + 3] = t.w;
        }
        const int cw = lane < DM ? lane : 0;
#pragma unroll
        for (int k = 0; k < DM; k += 4) {
            const float4 t = *reinterpret_cast<const float4 *>(A.W_o + (int64_t)cw * P.dp + k);
            wo[k] = t.x, wo[k + 1] = t.y, wo[k + 2] = t.z, wo[k + 3] = t.w;
        }
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < DM; ++k) acc = fmaf(o[k], wo[k], acc);
        float v = acc + A.b_o[lane];
        if (drop) v = u2gnn_keep(s1, (uint32_t)r, (uint32_t)lane, P.p) ? v * ks : 0.f;
        z1 = lane < P.d ? v + A.X[ro + lane] : 0.f;
        x1 = ln_row(z1, lane, P.d, P.eps, A.n1_w, A.n1_b, mu1, rs1);
#pragma unroll
        for (int k = 0; k < DM; ++k) xv[k] = __shfl(x1, k, 64);
    }
    if (writer) {
        A.Z1[ro + lane] = z1;   // dp == 64: one column per lane (padding columns and rows 0)
        A.X1[ro + lane] = x1;
        if (lane == 0) A.mean1[r] = mu1, A.rstd1[r] = rs1;
    }
    // a3.4: h = dropff(relu(x1 W1^T + b1)) over the hidden units, z2 partials = h W2^T
    float zp[DM];
#pragma unroll
    for (int k = 0; k < DM; ++k) zp[k] = 0.f;
    const uint32_t rkf = u2gnn_row_key(sff, (uint32_t)r);
    float *hrow = A.Hd + (int64_t)r * P.ffp;
    if constexpr (DIRECT) {
        for (int h = 64 * w + lane; h < P.ffp; h += 64 * LS_WAVES) {
            float w1[DM], w2[DM];
#pragma unroll
            for (int k = 0; k < DM; k += 4) {
                const float4 t = *reinterpret_cast<const float4 *>(A.W1 + (int64_t)h * P.dp + k);
                w1[k] = t.x, w1[k + 1] = t.y, w1[k + 2] = t.z, w1[k + 3] = t.w;
            }
#pragma unroll
            for (int k = 0; k < DM; ++k) w2[k] = A.W2[(int64_t)k * P.ffp + h];
            const bool keep = !drop || u2gnn_keep_rk(rkf, (uint32_t)h, thr);
            ffn_unit_fwd<DM>(xv, w1, w2, A.b1[h], keep, ks, live, hrow + h, zp);
        }
    } else {
        for (int h0 = 0; h0 < P.ffp; h0 += HC) {
            Stage<DM, HC, true> sg;
            sg.load(P, h0);
            __syncthreads();
            sg.store(w1s, w2s, b1s);
            __syncthreads();
#pragma unroll 4
            for (int u = 0; u < NU; ++u) {
                const int h = 64 * u + lane;
                if (h0 + h >= P.ffp) break;
                float w1[DM], w2[DM];
#pragma unroll
                for (int k = 0; k < DM; k += 4) {
                    const float4 t = *reinterpret_cast<const float4 *>(&w1s[h][k]);
                    w1[k] = t.x, w1[k + 1] = t.y, w1[k + 2] = t.z, w1[k + 3] = t.w;
                    const float4 q = *reinterpret_cast<const float4 *>(&w2s[h][k]);
                    w2[k] = q.x, w2[k + 1] = q.y, w2[k + 2] = q.z, w2[k + 3] = q.w;
                }
                const bool keep = !drop || u2gnn_keep_rk(rkf, (uint32_t)(h0 + h), thr);
                ffn_unit_fwd<DM>(xv, w1, w2, b1s[h], keep, ks, live, hrow + h0 + h, zp);
            }
        }
    }
#pragma unroll
    for (int k = 0; k < DM; ++k) zp[k] = wsum(zp[k]);
    if constexpr (DIRECT) {   // the 8 waves' partials, in wave order
        if (lane == 0)
#pragma unroll
            for (int k = 0; k < DM; ++k) xw[w][k] = zp[k];
        __syncthreads();
        if (w != 0) return;
#pragma unroll
        for (int k = 0; k < DM; ++k) {
            float t = xw[0][k];
#pragma unroll
            for (int y = 1; y < LS_WAVES; ++y) t += xw[y][k];
            zp[k] = t;
        }
    }
    float z2 = 0.f, x2 = 0.f, mu2 = 0.f, rs2 = 0.f;
    if (live) {
        float v = pick<DM>(zp, lane) + A.b2[lane];
        if (drop) v = u2gnn_keep(s2, (uint32_t)r, (uint32_t)lane, P.p) ? v * ks : 0.f;
        z2 = lane < P.d ? v + x1 : 0.f;
        x2 = ln_row(z2, lane, P.d, P.eps, A.n2_w, A.n2_b, mu2, rs2);
    }
    A.Z2[ro + lane] = z2;
    A.X2[ro + lane] = x2;
    if (lane == 0) A.mean2[r] = mu2, A.rstd2[r] = rs2;
}

// one hidden unit of the backward: dH = (Hd > 0) dF . W2[:, h] / (1-p), written; xp += dH W1[h]
template <int DM>
__device__ __forceinline__ void ffn_unit_bwd(const float (&fv)[DM], const float (&w1)[DM], const float (&w2)[DM], float hv,
                                             float ks, bool live, float *dst, float (&xp)[DM]) {
    float g = 0.f;
#pragma unroll
    for (int k = 0; k < DM; ++k) g = fmaf(fv[k], w2[k], g);
    g = (live && hv > 0.f) ? g * ks : 0.f;
    *dst = g;
#pragma unroll
    for (int k = 0; k < DM; ++k) xp[k] = fmaf(g, w1[k], xp[k]);
}

template <int DM, bool DIRECT>
__global__ void __launch_bounds__(LS_NT, ls_min_waves<DM>()) ls_bwd_kernel(LsP P) {
    constexpr int HC = DIRECT ? 64 : ls_hc<DM>(), NU = HC / 64;
    __shared__ __attribute__((aligned(16))) float w1s[DIRECT ? 1 : HC][DM];
    __shared__ __attribute__((aligned(16))) float w2s[DIRECT ? 1 : HC][DM];
    __shared__ float xw[DIRECT ? LS_WAVES : 1][DM];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r = ls_row<DIRECT>();
    const bool live = r < P.N;
    const bool writer = !DIRECT || w == 0;
    const u2gnn_small_tail_args &A = P.a;
    const bool drop = P.p > 0.f;
    const float ks = drop ? 1.f / (1.f - P.p) : 1.f;
    const uint64_t s1 = u2gnn_seed(P.s1, P.epoch), s2 = u2gnn_seed(P.s2, P.epoch);
    const int64_t ro = (int64_t)r * P.dp;
    // LayerNorm2^T: dz2 (residual branch, part of dX1) and dF = drop2'(dz2)
    float dz2 = 0.f, df = 0.f;
    float fv[DM];
#pragma unroll
    for (int k = 0; k < DM; ++k) fv[k] = 0.f;
    if (live) {
        dz2 = ln_row_bwd(A.dX2[ro + lane], A.Z2[ro + lane], A.mean2[r], A.rstd2[r], lane, P.d, A.n2_w);
        df = (drop && lane < P.d) ? (u2gnn_keep(s2, (uint32_t)r, (uint32_t)lane, P.p) ? dz2 * ks : 0.f) : dz2;
#pragma unroll
        for (int k = 0; k < DM; ++k) fv[k] = __shfl(df, k, 64);
    }
    if (writer) A.dF[ro + lane] = df;
    // FFN^T: dH = (Hd > 0) dF W2 / (1-p) over the hidden units, dX1 partials = dH W1
    float xp[DM];
#pragma unroll
    for (int k = 0; k < DM; ++k) xp[k] = 0.f;
    const float *hrow = A.Hd + (int64_t)r * P.ffp;
    float *dhrow = A.dH + (int64_t)r * P.ffp;
    if constexpr (DIRECT) {
        for (int h = 64 * w + lane; h < P.ffp; h += 64 * LS_WAVES) {
            float w1[DM], w2[DM];
#pragma unroll
            for (int k = 0; k < DM; k += 4) {
                const float4 t = *reinterpret_cast<const float4 *>(A.W1 + (int64_t)h * P.dp + k);
                w1[k] = t.x, w1[k + 1] = t.y, w1[k + 2] = t.z, w1[k + 3] = t.w;
            }
#pragma unroll
            for (int k = 0; k < DM; ++k) w2[k] = A.W2[(int64_t)k * P.ffp + h];
            ffn_unit_bwd<DM>(fv, w1, w2, hrow[h], ks, live, dhrow + h, xp);
        }
    } else {
        for (int h0 = 0; h0 < P.ffp; h0 += HC) {
            Stage<DM, HC, false> sg;
            sg.load(P, h0);
            float hvs[NU];   // this row's ReLU image of the chunk, loaded with the weights
#pragma unroll
            for (int u = 0; u < NU; ++u) hvs[u] = h0 + 64 * u + lane < P.ffp ? hrow[h0 + 64 * u + lane] : 0.f;
            __syncthreads();
            sg.store(w1s, w2s, nullptr);
            __syncthreads();
#pragma unroll 4
            for (int u = 0; u < NU; ++u) {
                const int h = 64 * u + lane;
                if (h0 + h >= P.ffp) break;
                float w1[DM], w2[DM];
#pragma unroll
                for (int k = 0; k < DM; k += 4) {
                    const float4 t = *reinterpret_cast<const float4 *>(&w1s[h][k]);
                    w1[k] = t.x, w1[k + 1] = t.y, w1[k + 2] = t.z, w1[k + 3] = t.w;
                    const float4 q = *reinterpret_cast<const float4 *>(&w2s[h][k]);
                    w2[k] = q.x, w2[k + 1] = q.y, w2[k + 2] = q.z, w2[k + 3] = q.w;
                }
                ffn_unit_bwd<DM>(fv, w1, w2, hvs[u], ks, live, dhrow + h0 + h, xp);
            }
        }
    }
#pragma unroll
    for (int k = 0; k < DM; ++k) xp[k] = wsum(xp[k]);
    if constexpr (DIRECT) {   // the 8 waves' partials, in wave order
        if (lane == 0)
#pragma unroll
            for (int k = 0; k < DM; ++k) xw[w][k] = xp[k];
        __syncthreads();
        if (w != 0) return;
#pragma unroll
        for (int k = 0; k < DM; ++k) {
            float t = xw[0][k];
#pragma unroll
            for (int y = 1; y < LS_WAVES; ++y) t += xw[y][k];
            xp[k] = t;
        }
    }
    float dx1 = 0.f, dz1 = 0.f, da = 0.f, dov = 0.f, dl = 0.f;
    if (live) {
        dx1 = lane < P.d ? dz2 + pick<DM>(xp, lane) : 0.f;
        // LayerNorm1^T: dX (residual branch) and dA = drop1'(dz1)
        dz1 = ln_row_bwd(dx1, A.Z1[ro + lane], A.mean1[r], A.rstd1[r], lane, P.d, A.n1_w);
        da = (drop && lane < P.d) ? (u2gnn_keep(s1, (uint32_t)r, (uint32_t)lane, P.p) ? dz1 * ks : 0.f) : dz1;
        // out-projection^T: dO_k = sum_c dA_c W_o[c][k], delta = rowsum(dO * O)
        float av[DM];
#pragma unroll
        for (int k = 0; k < DM; ++k) av[k] = __shfl(da, k, 64);
        const int kc = lane < DM ? lane : 0;
        float acc = 0.f;
#pragma unroll
        for (int c = 0; c < DM; ++c) acc = fmaf(av[c], A.W_o[(int64_t)c * P.dp + kc], acc);
        dov = lane < P.d ? acc : 0.f;
        dl = wsum(dov * A.O[ro + lane]);
    }
    A.dX1[ro + lane] = dx1;
    A.dX[ro + lane] = dz1;
    A.dA[ro + lane] = da;
    A.dO[ro + lane] = dov;
    if (lane == 0) A.delta[r] = dl;
}

int ls_dm(int64_t d) { return d < 1 ? 0 : d <= 24 ? (int)((d + 3) / 4 * 4) : d <= 32 ? 32 : 0; }

bool al16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

int ls_check(const u2gnn_small_tail_args *a, bool bwd) {
    if (!a || !ls_dm(a->d) || a->dp != 64 || a->n_valid < 1 || a->rows_pad < a->n_valid || (a->rows_pad % LS_WAVES) ||
        a->ff < 1 || a->ffp < a->ff || (a->ffp & 63) || a->p < 0.f || !(a->p < 1.f) || a->rows_pad > ((int64_t)1 << 30) ||
        a->ffp > ((int64_t)1 << 20))
        return U2GNN_E_ARG;
    const void *need[] = {a->W_o, a->b_o, a->n1_w, a->n1_b, a->W1, a->b1, a->W2, a->b2, a->n2_w, a->n2_b, a->O,
                          a->Z1, a->mean1, a->rstd1, a->Hd, a->Z2, a->mean2, a->rstd2};
    for (const void *q : need)
        if (!q) return U2GNN_E_ARG;
    if (!bwd && (!a->X || !a->X1 || !a->X2)) return U2GNN_E_ARG;
    if (bwd && (!a->dX2 || !a->dX1 || !a->dF || !a->dH || !a->dX || !a->dA || !a->dO || !a->delta)) return U2GNN_E_ARG;
    if (!al16(a->W_o) || !al16(a->W1) || !al16(a->O)) return U2GNN_E_ALIGN;
    return U2GNN_OK;
}

LsP ls_params(const u2gnn_small_tail_args *a) {
    LsP P;
    std::memset(&P, 0, sizeof(P));
    P.N = (int32_t)a->n_valid, P.Np = (int32_t)a->rows_pad, P.d = (int32_t)a->d, P.dp = (int32_t)a->dp;
    P.ff = (int32_t)a->ff, P.ffp = (int32_t)a->ffp, P.p = a->p, P.eps = a->eps;
    P.s1 = a->seed_drop1, P.sff = a->seed_dropff, P.s2 = a->seed_drop2, P.epoch = u2gnn_g_epoch;
    P.a = *a;
    return P;
}

// DIRECT below 1024 padded rows (fewer than 128 staged workgroups); the split changes only the order of the
// hidden-unit partial sums, so a run is deterministic either way
template <int DM>
int ls_launch(const LsP &P, bool bwd, hipStream_t st) {
    const bool direct = P.Np < 1024;
    const dim3 grid((unsigned)(direct ? P.Np : P.Np / LS_WAVES));
    if (bwd && direct) hipLaunchKernelGGL((ls_bwd_kernel<DM, true>), grid, dim3(LS_NT), 0, st, P);
    else if (bwd) hipLaunchKernelGGL((ls_bwd_kernel<DM, false>), grid, dim3(LS_NT), 0, st, P);
    else if (direct) hipLaunchKernelGGL((ls_fwd_kernel<DM, true>), grid, dim3(LS_NT), 0, st, P);
    else hipLaunchKernelGGL((ls_fwd_kernel<DM, false>), grid, dim3(LS_NT), 0, st, P);
    return u2gnn_launch_status();
}

int ls_run(const u2gnn_small_tail_args *a, bool bwd, void *stream) {
    const int rc = ls_check(a, bwd);
    if (rc != U2GNN_OK) return rc;
    const LsP P = ls_params(a);
    hipStream_t st = u2gnn_stream(stream);
    switch (ls_dm(a->d)) {
        case 4: return ls_launch<4>(P, bwd, st);
        case 8: return ls_launch<8>(P, bwd, st);
        case 12: return ls_launch<12>(P, bwd, st);
        case 16: return ls_launch<16>(P, bwd, st);
        case 20: return ls_launch<20>(P, bwd, st);
        case 24: return ls_launch<24>(P, bwd, st);
        default: return ls_launch<32>(P, bwd, st);
    }
}

}  // namespace

extern "C" {

int u2gnn_layer_tail_small_fwd(const u2gnn_small_tail_args *a, void *stream) { return ls_run(a, false, stream); }

int u2gnn_layer_tail_small_bwd(const u2gnn_small_tail_args *a, void *stream) { return ls_run(a, true, stream); }

}  // extern "C"
