// a3.3 + a3.4 forward of a mid-width encoder layer (32 < d <= 256, padded width dp = 64 CPL <= 256) over a few
// hundred rows -- torch.nn.TransformerEncoderLayer's out-projection + dropout1 + residual + LayerNorm1 and
// FFN (linear1 -> ReLU -> dropout -> linear2) + dropout2 + residual + LayerNorm2, post-LN
// (pytorch_U2GNN_Sup.py:19-21,35).
//
// C2 (IMDBBINARY, 4-graph batches of ~80 nodes: rows_pad = 128, dp = 128, ff = 1024) ran this as five launches
// of 4-6 us that each moved a few hundred KB (out-projection, LayerNorm1, FFN1, split-K FFN2, slab LayerNorm2):
// launch floors.  Here one launch does the row-local part and the existing slab pass finishes:
//   * workgroup (row block of MT_RB rows, hidden chunk of MT_HC units), 8 waves;
//   * the out-projection of the block's rows (O rows staged in LDS), dropout1, the residual and LayerNorm1 (block
//     reduction, two-pass) -- every chunk's workgroup forms them (a few KFLOP), the chunk-0 workgroup stores Z1,
//     X1, mean1, rstd1;
//   * FFN1 for the chunk's hidden units, ReLU, dropout, Hd stored;
//   * the chunk's FFN2 partial sums into slab `chunk`;
// then u2gnn_slab_bias_drop_resid_ln sums the chunk slabs and forms bias, dropout2, residual and LayerNorm2.
// Exact fp32 on the vector ALUs (per-lane fmaf partials, a fixed butterfly / block reduction order: deterministic), the same dropout
// hash (u2gnn_keep) as every other site.  Rows >= n_valid come out as zeros.
#include "u2gnn_common.h"

namespace {

#ifndef MT_NT_
#define MT_NT_ 512   // (-DMT_NT_=256: the 4-wave form, 20.6 vs 15.2 us per launch at C2)
#endif
constexpr int MT_NT = MT_NT_;   // threads (8 waves: one 16-row weight batch per wave and phase at dp = 128)
constexpr int MT_RB = 4;        // rows per workgroup (the butterfly reduces 16 weight rows x 4 rows)
constexpr int MT_HC = 128;      // hidden units per workgroup

struct MtP {
    u2gnn_small_tail_args a;
    float *slabs;    // [nchunk][rows_pad][dp]
    const uint64_t *epoch;
};

__device__ __forceinline__ float4 mt_ld4(const float *p) { return *reinterpret_cast<const float4 *>(p); }

static_assert(MT_RB == 4, "the butterfly below reduces 16 weight rows x 4 activation rows = 64 outputs per wave");

// 16 weight rows W[i0 + i] (stride ldw; row elements k < klim, the rest and rows i >= valid read as 0) against the
// MT_RB activation rows xs (LDS, stride ldx), lanes along k (element k = lane + 64 m): every weight load is one
// coalesced 256-byte wave access and all 16 CPLK of them are in flight together.  The 64 per-lane partial sums
// (output o = 4 i + r) are reduced by one transpose butterfly -- at step s the lanes with bit 5-s set keep the
// upper half of their outputs and trade the lower half with lane ^ (32 >> s): 63 shuffles instead of 64 wave
// sums -- after which lane l holds output l complete.  Fixed order: deterministic.
// The 16 weight rows of one batch, loaded ahead of their phase (round 6): every load unconditional from a clamped
// address (rows i >= valid and elements k >= klim read a valid word and are zeroed at use), so a kernel can issue
// all its phases' weights with the first loads and pay one memory round trip instead of one per phase
template <int CPLK>
struct W16 {
    float v[16][CPLK];
    int valid, klim;
    __device__ __forceinline__ void load(const float *W, int64_t ldw, int i0, int valid_, int klim_, int lane) {
        valid = valid_, klim = klim_;
        const int il = valid_ > 0 ? valid_ - 1 : 0, kl = klim_ > 0 ? klim_ - 1 : 0;
#pragma unroll
        for (int i = 0; i < 16; ++i)
#pragma unroll
            for (int m = 0; m < CPLK; ++m) v[i][m] = W[(int64_t)(i0 + min(i, il)) * ldw + min(lane + 64 * m, kl)];
    }
};

template <int CPLK>
__device__ __forceinline__ float dot16x4w(const W16<CPLK> &W, const float *xs, int ldx, int lane) {
    float wv[16][CPLK];
#pragma unroll
    for (int i = 0; i < 16; ++i)
#pragma unroll
        for (int m = 0; m < CPLK; ++m) wv[i][m] = (i < W.valid && lane + 64 * m < W.klim) ? W.v[i][m] : 0.f;
    float xv[MT_RB][CPLK];
#pragma unroll
    for (int r = 0; r < MT_RB; ++r)
#pragma unroll
        for (int m = 0; m < CPLK; ++m) xv[r][m] = xs[r * ldx + lane + 64 * m];
    float v[64];
#pragma unroll
    for (int i = 0; i < 16; ++i)
#pragma unroll
        for (int r = 0; r < MT_RB; ++r) {
            float a = 0.f;
#pragma unroll
            for (int m = 0; m < CPLK; ++m) a = fmaf(xv[r][m], wv[i][m], a);
            v[4 * i + r] = a;
        }
#pragma unroll
    for (int st = 0; st < 6; ++st) {
        const int o = 32 >> st, n = 64 >> st;
        const bool up = (lane & o) != 0;
#pragma unroll
        for (int i = 0; i < n / 2; ++i) {
            const float send = up ? v[i] : v[i + n / 2];
            const float keep = up ? v[i + n / 2] : v[i];
            v[i] = keep + __shfl_xor(send, o, 64);
        }
    }
    return v[0];
}

template <int CPLK>
__device__ __forceinline__ float dot16x4(const float *W, int64_t ldw, int i0, int valid, int klim, const float *xs,
                                         int ldx, int lane) {
    W16<CPLK> w;
    w.load(W, ldw, i0, valid, klim, lane);
    return dot16x4w<CPLK>(w, xs, ldx, lane);
}

// the waves' partial sums of one row in a fixed pairwise order
template <int NW> __device__ __forceinline__ float wsum_fixed(const float *p) {
    float a[NW];
#pragma unroll
    for (int i = 0; i < NW; ++i) a[i] = p[i];
#pragma unroll
    for (int h = NW / 2; h > 0; h >>= 1)
#pragma unroll
        for (int i = 0; i < h; ++i) a[i] += a[i + h];
    return a[0];
}

template <int CPL>
__global__ void __launch_bounds__(MT_NT) mid_tail_fwd_kernel(MtP P) {
    constexpr int DP = 64 * CPL;
    constexpr int NW = MT_NT / 64;                                    // waves
    __shared__ __attribute__((aligned(16))) float os[MT_RB][DP];     // O rows
    __shared__ __attribute__((aligned(16))) float zs[MT_RB][DP];     // Z1 rows
    __shared__ __attribute__((aligned(16))) float xs[MT_RB][DP];     // X1 rows
    __shared__ __attribute__((aligned(16))) float hs[MT_RB][MT_HC];  // the chunk's hidden activations
    __shared__ float red[MT_RB][NW];
    const u2gnn_small_tail_args &A = P.a;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int r0 = (int)blockIdx.x * MT_RB, ch = (int)blockIdx.y;
    const int N = (int)A.n_valid, d = (int)A.d, ffp = (int)A.ffp;
    const int64_t rows_pad = A.rows_pad;
    const bool drop = A.p > 0.f;
    const float ks = drop ? 1.f / (1.f - A.p) : 1.f;
    const uint32_t thr = u2gnn_keep_thr(A.p);
    const uint64_t s1 = u2gnn_seed(A.seed_drop1, P.epoch), sff = u2gnn_seed(A.seed_dropff, P.epoch);
    const int lr = lane & 3, li = lane >> 2;   // the (activation row, weight row) of this lane's butterfly output
    const int h0 = ch * MT_HC, nu = min(MT_HC, ffp - h0);
    // every global operand of the wave's first batch in each phase, issued together with the O rows (round 6: the
    // phases' weight, bias and residual loads were seven dependent memory round trips, tools/isa_waits.py)
    // (dp <= 128: the three weight batches fit the registers; wider rows load each batch at its phase)
    constexpr bool PF = CPL <= 2;
    W16<CPL> wo_p, w1_p;
    W16<MT_HC / 64> w2_p;
    if constexpr (PF) {
        wo_p.load(A.W_o, DP, 16 * w, d - 16 * w, DP, lane);
        w1_p.load(A.W1, DP, h0 + 16 * w, nu - 16 * w, DP, lane);
        w2_p.load(A.W2 + h0, ffp, 16 * w, DP - 16 * w, nu, lane);
    }
    const float bo_p = A.b_o[min(16 * w + li, DP - 1)], x_p = A.X[(int64_t)(r0 + lr) * DP + min(16 * w + li, DP - 1)];
    const float b1_p = A.b1[min(h0 + 16 * w + li, ffp - 1)];
    const float g1 = A.n1_w[min(t, d - 1)], b1n = A.n1_b[min(t, d - 1)];
    for (int e = t; e < MT_RB * DP / 4; e += MT_NT) {
        const int r = e / (DP / 4), k = 4 * (e % (DP / 4));
        *reinterpret_cast<float4 *>(&os[r][k]) = mt_ld4(A.O + (int64_t)(r0 + r) * DP + k);
    }
    __syncthreads();
    // a3.3: z1[c] = drop1(sum_k O[k] W_o[c][k] + b_o[c]) + x[c]; wave w takes the 16-column batches w, w + NW, ...
    for (int b = w; b < DP / 16; b += NW) {
        const int c = 16 * b + li, row = r0 + lr;
        const bool first = b == w;   // (bias and residual prefetched; the weights too when PF)
        float v = (PF && first) ? dot16x4w<CPL>(wo_p, &os[0][0], DP, lane)
                        : dot16x4<CPL>(A.W_o, DP, 16 * b, d - 16 * b, DP, &os[0][0], DP, lane);
        float z = 0.f;
        if (c < d && row < N) {
            v += first ? bo_p : A.b_o[c];
            if (drop) v = u2gnn_keep(s1, (uint32_t)row, (uint32_t)c, A.p) ? v * ks : 0.f;
            z = v + (first ? x_p : A.X[(int64_t)row * DP + c]);
        }
        zs[lr][c] = z;
    }
    __syncthreads();
    // LayerNorm1 over the first d columns: mean, then the mean square deviation (block reductions, fixed order);
    // thread t holds column t
    const int c = t;
    float z[MT_RB], mu[MT_RB], rs[MT_RB];
#pragma unroll
    for (int r = 0; r < MT_RB; ++r) {
        z[r] = c < DP ? zs[r][c] : 0.f;
        const float s = wave_sum(z[r]);
        if (lane == 0) red[r][w] = s;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < MT_RB; ++r) mu[r] = wsum_fixed<NW>(red[r]) / (float)d;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < MT_RB; ++r) {
        const float dv = c < d ? z[r] - mu[r] : 0.f;
        const float s = wave_sum(dv * dv);
        if (lane == 0) red[r][w] = s;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < MT_RB; ++r)
        rs[r] = rsqrtf(wsum_fixed<NW>(red[r]) / (float)d + A.eps);
#pragma unroll
    for (int r = 0; r < MT_RB; ++r) {
        const int row = r0 + r;
        const bool live = row < N;
        const float x1 = (live && c < d) ? (z[r] - mu[r]) * rs[r] * g1 + b1n : 0.f;   // (g1, b1n: column t's)
        if (c < DP) {
            xs[r][c] = x1;
            if (ch == 0) {
                A.Z1[(int64_t)row * DP + c] = z[r];
                A.X1[(int64_t)row * DP + c] = x1;
            }
        }
        if (ch == 0 && c == 0) {
            A.mean1[row] = live ? mu[r] : 0.f;
            A.rstd1[row] = live ? rs[r] : 0.f;
        }
    }
    __syncthreads();
    // a3.4 FFN1: h_j = dropff(relu(sum_k x1[k] W1[j][k] + b1[j])) for the chunk's units j, 16-unit batches
    for (int b = w; b < MT_HC / 16; b += NW) {
        const int u = 16 * b + li, j = h0 + u, row = r0 + lr;
        const bool first = b == w;
        float h = (PF && first) ? dot16x4w<CPL>(w1_p, &xs[0][0], DP, lane)
                        : dot16x4<CPL>(A.W1, DP, h0 + 16 * b, nu - 16 * b, DP, &xs[0][0], DP, lane);
        if (u < nu && row < N) {
            h = fmaxf(h + (first ? b1_p : A.b1[j]), 0.f);
            if (drop) h = u2gnn_keep_rk(u2gnn_row_key(sff, (uint32_t)row), (uint32_t)j, thr) ? h * ks : 0.f;
        } else {
            h = 0.f;
        }
        hs[lr][u] = h;
    }
    __syncthreads();
    // Hd of the chunk, coalesced: thread t -> (row, 4 units)
    for (int e = t; e < MT_RB * MT_HC / 4; e += MT_NT) {
        const int r = e / (MT_HC / 4), u = 4 * (e % (MT_HC / 4));
        if (u < nu)
            *reinterpret_cast<float4 *>(A.Hd + (int64_t)(r0 + r) * ffp + h0 + u) =
                *reinterpret_cast<const float4 *>(&hs[r][u]);
    }
    // the chunk's FFN2 partial sums: column c gets sum over the chunk's units of h_u W2[c][h0 + u], 16-column
    // batches, lanes along the units
    for (int b = w; b < DP / 16; b += NW) {
        const int cc = 16 * b + li;
        const float v = (PF && b == w) ? dot16x4w<MT_HC / 64>(w2_p, &hs[0][0], MT_HC, lane)
                               : dot16x4<MT_HC / 64>(A.W2 + h0, ffp, 16 * b, DP - 16 * b, nu, &hs[0][0], MT_HC, lane);
        P.slabs[((int64_t)ch * rows_pad + r0 + lr) * DP + cc] = v;
    }
}

bool al16(const void *p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

extern "C" {

int64_t u2gnn_layer_tail_mid_ws_floats(int64_t rows_pad, int64_t dp, int64_t ffp) {
    if (rows_pad < 0 || dp < 64 || dp > 256 || dp % 64 || ffp < 64 || ffp % 64) return -1;
    return (ffp + MT_HC - 1) / MT_HC * rows_pad * dp;
}

int u2gnn_layer_tail_mid_fwd(const u2gnn_small_tail_args *t, float *ws, int64_t ws_floats, void *stream) {
    if (!t) return U2GNN_E_ARG;
    const u2gnn_small_tail_args &a = *t;
    if (a.d < 1 || a.dp != (a.d + 63) / 64 * 64 || a.dp > 256 || a.n_valid < 1 || a.rows_pad < a.n_valid ||
        a.rows_pad % MT_RB || a.ff < 1 || a.ffp < a.ff || a.ffp % 64 || !(a.p < 1.f) || a.p < 0.f)
        return U2GNN_E_ARG;
    const float *in[] = {a.W_o, a.b_o, a.n1_w, a.n1_b, a.W1, a.b1, a.W2, a.b2, a.n2_w, a.n2_b, a.O, a.X};
    for (const float *q : in)
        if (!q) return U2GNN_E_ARG;
    float *out[] = {a.Z1, a.X1, a.mean1, a.rstd1, a.Hd, a.Z2, a.X2, a.mean2, a.rstd2};
    for (const float *q : out)
        if (!q) return U2GNN_E_ARG;
    if (!al16(a.W_o) || !al16(a.W1) || !al16(a.W2) || !al16(a.O) || !al16(ws)) return U2GNN_E_ALIGN;
    const int64_t need = u2gnn_layer_tail_mid_ws_floats(a.rows_pad, a.dp, a.ffp);
    if (!ws || need < 0 || ws_floats < need) return U2GNN_E_ARG;
    MtP P;
    P.a = a;
    P.slabs = ws;
    P.epoch = u2gnn_cur_epoch();
    const int nchunk = (int)((a.ffp + MT_HC - 1) / MT_HC);
    const dim3 grid((unsigned)(a.rows_pad / MT_RB), (unsigned)nchunk);
    hipStream_t st = u2gnn_stream(stream);
    switch (a.dp / 64) {
        case 1: hipLaunchKernelGGL(mid_tail_fwd_kernel<1>, grid, dim3(MT_NT), 0, st, P); break;
        case 2: hipLaunchKernelGGL(mid_tail_fwd_kernel<2>, grid, dim3(MT_NT), 0, st, P); break;
        case 3: hipLaunchKernelGGL(mid_tail_fwd_kernel<3>, grid, dim3(MT_NT), 0, st, P); break;
        default: hipLaunchKernelGGL(mid_tail_fwd_kernel<4>, grid, dim3(MT_NT), 0, st, P); break;
    }
    const int rc = u2gnn_launch_status();
    if (rc != U2GNN_OK) return rc;
    // LayerNorm2 from the chunk slabs: bias, dropout2, residual X1
    return u2gnn_slab_bias_drop_resid_ln(ws, nchunk, a.rows_pad * a.dp, a.dp, a.b2, a.X1, a.dp, a.p, a.seed_drop2, a.Z2,
                                         a.dp, a.n2_w, a.n2_b, a.X2, a.dp, a.mean2, a.rstd2, a.d, a.n_valid, a.rows_pad,
                                         a.eps, stream);
}

}  // extern "C"
