// Shared pieces of the U2GNN GEMM kernels (gemm.hip: fp32-operand kernels; gemm_x2.hip: kernels over
// pre-split bf16 hi/lo operands): kernel parameters, the fused epilogues and the XCD-aware tile map.
#pragma once
#include "u2gnn_common.h"

// kernel parameters (shared by both translation units, hence outside the anonymous namespace)
struct GemmP {
    const float *A;
    const float *B;
    float *C;
    int64_t lda, ldb, ldc;
    int32_t M, N, K;  // K = per-split depth (multiple of the K tile)
    int32_t Ktot;     // full depth; split z covers [z*K, min((z+1)*K, Ktot))
    int32_t gm, gn;
    int64_t slab_stride;
    const float *bias;
    const float *aux0;
    const float *aux1;
    const float *rowvec;
    int64_t ld_aux;
    float alpha;
    int32_t scale_cols;
    float p;
    uint64_t seed;
    const uint32_t *keep;
    int64_t ld_keep;
    // x2 output (U2GNN x2 format: per 8 columns hi then lo bf16, see u2gnn_hip.h)
    __bf16 *Cx2;          // non-null: the epilogue also writes C in x2 format
    int64_t ldcx2;        // bf16 elements
    int32_t cx2_col0;     // Cx2 receives columns >= cx2_col0 only
    float cx2_h3;         // 0: bf16 x2; > 0 (f16x3 kind): fp16 hi / lo of cx2_h3 * C (u2gnn_hip.h U2GNN_H3_X2_EXP)
    int32_t n_valid;   // STORE_ROWSTAT: real keys (columns >= n_valid are masked)
    const uint64_t *epoch;      // seed epoch at launch (u2gnn_set_seed_epoch): seed ^= *epoch * golden
    // EPI_BIAS_DROP_RESID_LN: the post-LayerNorm of the row-complete 64-column result
    const float *ln_gamma, *ln_beta;
    float *ln_y, *ln_mean, *ln_rstd;
    int64_t ln_ldy;
    int32_t ln_d, ln_rows;
    float ln_eps;
    // EPI_STORE_ROWDOT: per-64-column-group row partials of C*aux0; EPI_DS_SIGNED_PARTS: rowvec_parts of them
    float *rowpart;
    int64_t ld_rowpart;
    int32_t rowvec_parts;
    int64_t ld_rowvec;
    float h3_sa, h3_sb, h3_inv;   // f16x3: operand pre-scales 2^h3_exp_a, 2^h3_exp_b and the result's 2^-(sum)
};


namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// Internal epilogue template code (not an ABI value): ATTN_DS_SIGNED with delta given as rowvec_parts
// STORE_ROWDOT partials.  A separate instantiation, so that the plain ATTN_DS_SIGNED kernel (the C4
// dS product) keeps its registers and schedule: carrying the partials there cost it ~10 % (113 -> 124 us).
constexpr int EPI_DS_SIGNED_PARTS = 100;
template <int EPI> constexpr bool ds_signed = EPI == U2GNN_EPI_ATTN_DS_SIGNED || EPI == EPI_DS_SIGNED_PARTS;



// four consecutive columns (col % 4 == 0) of one row; every vector operand is 16-byte aligned
// with a leading dimension that is a multiple of 4 (checked by u2gnn_gemm)
__device__ __forceinline__ float4 ld4(const float *p) { return *reinterpret_cast<const float4 *>(p); }

// The epilogue runs in two passes per 32-row slice of a wave's tile: epi_fetch issues every
// auxiliary load (P, keep words, residual, bias, C) first, then epilogue4 combines and stores.
// Interleaved in one loop, each load would sit behind the previous store (the compiler cannot
// prove C distinct from the aux operands) and the slice would pay one memory round trip per
// 4 columns.
template <int EPI>
__device__ __forceinline__ void epi_fetch(const GemmP &P, int row, int col, float4 &a, float4 &b, uint32_t &kb) {
    if constexpr (ds_signed<EPI>) {
        a = ld4(P.aux0 + (int64_t)row * P.ld_aux + col);
    } else if constexpr (EPI == U2GNN_EPI_ATTN_DS) {
        const int64_t o = (int64_t)row * P.ld_aux + col;
        a = ld4(P.aux0 + o);
        if (P.keep)
            kb = P.keep[(int64_t)row * P.ld_keep + (col >> 5)] >> (col & 31);
        else
            b = ld4(P.aux1 + o);
    } else if constexpr (EPI == U2GNN_EPI_ACCUM) {
        a = ld4(P.C + (int64_t)row * P.ldc + col);
    } else if constexpr (EPI == U2GNN_EPI_RELU_DROP_BWD || EPI == U2GNN_EPI_STORE_ROWDOT) {
        a = ld4(P.aux0 + (int64_t)row * P.ld_aux + col);
    } else if constexpr (EPI != U2GNN_EPI_STORE) {   // bias epilogues
        a = ld4(P.bias + col);
        if constexpr (EPI == U2GNN_EPI_BIAS_DROP_RESID) b = ld4(P.aux0 + (int64_t)row * P.ld_aux + col);
    }
}

// four consecutive columns (col % 4 == 0) of one row; a, b, kb, dl = what epi_fetch loaded
template <int EPI>
__device__ __forceinline__ float4 epilogue4(const GemmP &P, int row, int col, float4 v, float4 a, float4 b,
                                            uint32_t kb, float dl) {
    if constexpr (EPI == U2GNN_EPI_STORE_ROWSTAT) {
        // masked keys (columns >= n_valid) stored as -inf: their probability is exp(-inf) = 0 downstream
        const float ni = -INFINITY;
        return make_float4(col < P.n_valid ? P.alpha * v.x : ni, col + 1 < P.n_valid ? P.alpha * v.y : ni,
                           col + 2 < P.n_valid ? P.alpha * v.z : ni, col + 3 < P.n_valid ? P.alpha * v.w : ni);
    } else if constexpr (EPI == U2GNN_EPI_STORE || EPI == U2GNN_EPI_STORE_ROWDOT) {
        return make_float4(P.alpha * v.x, P.alpha * v.y, P.alpha * v.z, P.alpha * v.w);
    } else if constexpr (ds_signed<EPI>) {
        // x = Pd = P/(1-p) where kept (sign clear), x = -P where dropped (sign set):
        // dS = P*(keep*dPd/(1-p) - delta) = kept ? x*(dPd - (1-p)*delta) : x*delta
        const float q = (1.f - P.p) * dl;
        const float x[4] = {a.x, a.y, a.z, a.w}, g[4] = {v.x, v.y, v.z, v.w};
        float o[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) o[c] = x[c] * ((__float_as_uint(x[c]) >> 31) ? dl : g[c] - q);
        return make_float4(o[0], o[1], o[2], o[3]);
    } else if constexpr (EPI == U2GNN_EPI_ATTN_DS) {
        const float4 pr = a;
        if (P.keep) {   // dS = P * (keep * dPd / (1-p) - delta): 4 keep bits instead of 16 B of Pd
            const float s = 1.f / (1.f - P.p);
            return make_float4(pr.x * (((kb & 1u) ? v.x * s : 0.f) - dl), pr.y * (((kb & 2u) ? v.y * s : 0.f) - dl),
                               pr.z * (((kb & 4u) ? v.z * s : 0.f) - dl), pr.w * (((kb & 8u) ? v.w * s : 0.f) - dl));
        }
        const float4 pd = b;
        return make_float4(pd.x * v.x - pr.x * dl, pd.y * v.y - pr.y * dl, pd.z * v.z - pr.z * dl,
                           pd.w * v.w - pr.w * dl);
    } else if constexpr (EPI == U2GNN_EPI_ACCUM) {
        const float4 c = a;
        return make_float4(c.x + P.alpha * v.x, c.y + P.alpha * v.y, c.z + P.alpha * v.z, c.w + P.alpha * v.w);
    } else if constexpr (EPI == U2GNN_EPI_RELU_DROP_BWD) {
        const float4 h = a;
        const float s = 1.f / (1.f - P.p);
        return make_float4(h.x > 0.f ? v.x * s : 0.f, h.y > 0.f ? v.y * s : 0.f, h.z > 0.f ? v.z * s : 0.f,
                           h.w > 0.f ? v.w * s : 0.f);
    } else {  // bias epilogues: per-column dropout hash
        float x[4] = {v.x + a.x, v.y + a.y, v.z + a.z, v.w + a.w};
        if constexpr (EPI == U2GNN_EPI_BIAS) {
#pragma unroll
            for (int c = 0; c < 4; ++c) x[c] = col + c < P.scale_cols ? x[c] * P.alpha : x[c];
        } else {
            if constexpr (EPI == U2GNN_EPI_BIAS_RELU_DROP) {
#pragma unroll
                for (int c = 0; c < 4; ++c) x[c] = fmaxf(x[c], 0.f);
            }
            if (P.p > 0.f) {
                // col % 4 == 0: the four columns are two hash pairs
                const float s = 1.f / (1.f - P.p);
                const uint32_t rk = u2gnn_row_key(P.seed, (uint32_t)row), thr = u2gnn_keep_thr(P.p);
                const uint32_t h0 = u2gnn_pair_hash(rk, (uint32_t)col >> 1), h1 = u2gnn_pair_hash(rk, ((uint32_t)col >> 1) + 1);
                const bool kp[4] = {u2gnn_keep_lo(h0, thr), u2gnn_keep_hi(h0, thr), u2gnn_keep_lo(h1, thr),
                                    u2gnn_keep_hi(h1, thr)};
#pragma unroll
                for (int c = 0; c < 4; ++c) x[c] = kp[c] ? x[c] * s : 0.f;
            }
            if constexpr (EPI == U2GNN_EPI_BIAS_DROP_RESID) {
                x[0] += b.x, x[1] += b.y, x[2] += b.z, x[3] += b.w;
            }
        }
        return make_float4(x[0], x[1], x[2], x[3]);
    }
}

// The attention backward's delta of one row: rowvec[row], or (ABI v8) the sum of the dO GEMM's
// STORE_ROWDOT partials (one per 64 columns) in group order -- one fixed order, so the native and
// Python paths agree.  The partials are loaded into registers with the other epilogue operands and
// summed only when the slice is stored: summing at load time would make the wave wait for every load
// issued before them (the dS kernel prefetches slice 0's P tile ahead of its main loop).
constexpr int DELTA_REGS = 8;
struct DeltaParts {
    float v[DELTA_REGS];
};
__device__ __forceinline__ void delta_load(const GemmP &P, int row, DeltaParts &d) {
    if (P.rowvec_parts <= 1) {
        d.v[0] = P.rowvec[row];
        return;
    }
#pragma unroll
    for (int q = 0; q < DELTA_REGS; ++q)
        d.v[q] = q < P.rowvec_parts ? P.rowvec[(int64_t)q * P.ld_rowvec + row] : 0.f;
}
__device__ __forceinline__ float delta_sum(const GemmP &P, int row, const DeltaParts &d) {
    if (P.rowvec_parts <= 1) return d.v[0];
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < DELTA_REGS; ++q)
        if (q < P.rowvec_parts) s += d.v[q];
    for (int q = DELTA_REGS; q < P.rowvec_parts; ++q) s += P.rowvec[(int64_t)q * P.ld_rowvec + row];
    return s;
}

// lane (li, kh) of MFMA tile (i, j) holds C[row = li][cols 8g + 4kh .. +3] in acc[i][j][4g .. 4g+3].
// One 32-row slice (fixed i) of a wave's tile: its auxiliary operands, then its stores.
template <int EPI, int TN>
struct EpiSlice {
    float4 a[TN][4], b[TN][4];
    uint32_t kb[TN][4];
    float dl;
    DeltaParts dp;    // EPI_DS_SIGNED_PARTS: dl = delta_sum(dp) when the slice is stored
};

template <int EPI, int TN>
__device__ __forceinline__ void fetch_slice(const GemmP &P, int row, int c0, int kh, EpiSlice<EPI, TN> &e) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            e.a[j][g] = e.b[j][g] = make_float4(0.f, 0.f, 0.f, 0.f);
            e.kb[j][g] = 0;
            epi_fetch<EPI>(P, row, c0 + j * 32 + 8 * g + 4 * kh, e.a[j][g], e.b[j][g], e.kb[j][g]);
        }
    e.dl = (EPI == U2GNN_EPI_ATTN_DS || EPI == U2GNN_EPI_ATTN_DS_SIGNED) ? P.rowvec[row] : 0.f;
    if constexpr (EPI == EPI_DS_SIGNED_PARTS) delta_load(P, row, e.dp);
}

// One slice's stores.  STORE_ROWDOT: returns this lane's share of sum_n C[row,n] * aux0[row,n] over
// the wave's columns (TN MFMA tiles in j order, columns 8g + 4kh of each), 0 otherwise.
template <int EPI, int TM, int TN>
__device__ __forceinline__ float store_slice(const GemmP &P, float *C, const f32x16 (&acc)[TM][TN], int i, int row,
                                             int c0, int kh, const EpiSlice<EPI, TN> &e) {
    float dl = e.dl;
    if constexpr (EPI == EPI_DS_SIGNED_PARTS) dl = delta_sum(P, row, e.dp);
    float rs = 0.f;
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int col = c0 + j * 32 + 8 * g + 4 * kh;
            const float4 v = make_float4(acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2],
                                         acc[i][j][4 * g + 3]);
            const float4 o = epilogue4<EPI>(P, row, col, v, e.a[j][g], e.b[j][g], e.kb[j][g], dl);
            if (P.C) *reinterpret_cast<float4 *>(C + (int64_t)row * P.ldc + col) = o;
            if (P.Cx2 && col >= P.cx2_col0) {
                if (P.cx2_h3 > 0.f) store_x2h_4(P.Cx2, P.ldcx2, row, col, o, P.cx2_h3);
                else store_x2_4(P.Cx2, P.ldcx2, row, col, o);
            }
            if constexpr (EPI == U2GNN_EPI_STORE_ROWDOT) {
                const float4 x = e.a[j][g];
                rs += o.x * x.x + o.y * x.y + o.z * x.z + o.w * x.w;
            }
        }
    return rs;
}

// Attention dS with keep bits: slice 0's P tile, keep words and delta fetched before the main loop
// (TN*16 + TN + 1 VGPRs), so they land under the MFMAs and the epilogue pays one round trip less.
template <int TN>
struct PreDS {
    float4 p[TN][4];
    uint32_t kw[TN];
    float dl;
    DeltaParts dp;
};

template <int EPI, int TN>
__device__ __forceinline__ void prefetch_ds(const GemmP &P, int row, int c0, int kh, PreDS<TN> &f) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        f.kw[j] = EPI == U2GNN_EPI_ATTN_DS ? P.keep[(int64_t)row * P.ld_keep + ((c0 + j * 32) >> 5)] : 0u;
#pragma unroll
        for (int g = 0; g < 4; ++g) f.p[j][g] = ld4(P.aux0 + (int64_t)row * P.ld_aux + c0 + j * 32 + 8 * g + 4 * kh);
    }
    if constexpr (EPI == EPI_DS_SIGNED_PARTS) delta_load(P, row, f.dp);
    else f.dl = P.rowvec[row];
}

template <int EPI, int TN>
__device__ __forceinline__ void slice_from_pre(const PreDS<TN> &pre, int kh, EpiSlice<EPI, TN> &e) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            e.a[j][g] = pre.p[j][g];
            e.b[j][g] = make_float4(0.f, 0.f, 0.f, 0.f);
            e.kb[j][g] = pre.kw[j] >> ((8 * g + 4 * kh) & 31);
        }
    e.dl = pre.dl;
    e.dp = pre.dp;
}

// EPI_BIAS_DROP_RESID_LN on 64 x 64 blocks of 2 x 2 waves that cover whole 64-column rows: the
// bias-dropout-residual result Z is stored as usual and kept in registers, then each row's LayerNorm
// (two-pass: mean, then the mean square deviation, over the first ln_d columns) is reduced across the
// row's two lanes (l, l ^ 32) and its two waves (LDS), and Y = (Z - mean) * rstd * gamma + beta is
// written with the row's mean / rstd -- the separate layernorm_fwd launch of a d <= 64 encoder.
template <int TM, int TN>
__device__ __forceinline__ void store_tile_ln(const GemmP &P, float *C, const f32x16 (&acc)[TM][TN], int r0, int c0,
                                              int li, int kh, const EpiSlice<U2GNN_EPI_BIAS_DROP_RESID, TN> *pa) {
    static_assert(TM == 1 && TN == 1, "row-complete LayerNorm epilogue: 64 x 64 blocks of 2 x 2 waves");
    constexpr int E = U2GNN_EPI_BIAS_DROP_RESID;
    __shared__ float lnred[2][2][64];
    const int row = r0 + li;
    const int rb = (r0 & 63) + li, wn = (c0 & 63) >> 5;
    EpiSlice<E, TN> e;
    if (pa) e = *pa;
    else fetch_slice<E>(P, row, c0, kh, e);
    float z[16];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const int col = c0 + 8 * g + 4 * kh;
        const float4 v = make_float4(acc[0][0][4 * g], acc[0][0][4 * g + 1], acc[0][0][4 * g + 2], acc[0][0][4 * g + 3]);
        const float4 o = epilogue4<E>(P, row, col, v, e.a[0][g], e.b[0][g], e.kb[0][g], e.dl);
        if (P.C) *reinterpret_cast<float4 *>(C + (int64_t)row * P.ldc + col) = o;
        z[4 * g] = o.x, z[4 * g + 1] = o.y, z[4 * g + 2] = o.z, z[4 * g + 3] = o.w;
    }
    const int d = P.ln_d;
    float gm[16], bt[16];
    // unpadded [d] vectors: float4 loads of full 4-column chunks when 16-byte aligned (the flat
    // parameter buffer's views are), clamped element loads otherwise
    const bool gb16 = ((reinterpret_cast<uintptr_t>(P.ln_gamma) | reinterpret_cast<uintptr_t>(P.ln_beta)) & 15) == 0;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const int col0 = c0 + 8 * g + 4 * kh;
        if (gb16 && col0 + 4 <= d) {
            const float4 gv = ld4(P.ln_gamma + col0), bv = ld4(P.ln_beta + col0);
            gm[4 * g] = gv.x, gm[4 * g + 1] = gv.y, gm[4 * g + 2] = gv.z, gm[4 * g + 3] = gv.w;
            bt[4 * g] = bv.x, bt[4 * g + 1] = bv.y, bt[4 * g + 2] = bv.z, bt[4 * g + 3] = bv.w;
            continue;
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int col = col0 + c;
            const int cc = col < d ? col : d - 1;
            gm[4 * g + c] = P.ln_gamma[cc];
            bt[4 * g + c] = P.ln_beta[cc];
        }
    }
    float s = 0.f;
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int c = 0; c < 4; ++c) s += (c0 + 8 * g + 4 * kh + c < d) ? z[4 * g + c] : 0.f;
    s += __shfl_xor(s, 32, 64);
    if (kh == 0) lnred[0][wn][rb] = s;
    __syncthreads();
    const float mu = (lnred[0][0][rb] + lnred[0][1][rb]) / (float)d;
    float q = 0.f;
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const float t = (c0 + 8 * g + 4 * kh + c < d) ? z[4 * g + c] - mu : 0.f;
            q += t * t;
        }
    q += __shfl_xor(q, 32, 64);
    if (kh == 0) lnred[1][wn][rb] = q;
    __syncthreads();
    const float rs = rsqrtf((lnred[1][0][rb] + lnred[1][1][rb]) / (float)d + P.ln_eps);
    const bool live = row < P.ln_rows;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const int col = c0 + 8 * g + 4 * kh;
        float y[4];
#pragma unroll
        for (int c = 0; c < 4; ++c)
            y[c] = (live && col + c < d) ? (z[4 * g + c] - mu) * rs * gm[4 * g + c] + bt[4 * g + c] : 0.f;
        *reinterpret_cast<float4 *>(P.ln_y + (int64_t)row * P.ln_ldy + col) = make_float4(y[0], y[1], y[2], y[3]);
    }
    if (kh == 0 && wn == 0) {
        P.ln_mean[row] = live ? mu : 0.f;
        P.ln_rstd[row] = live ? rs : 0.f;
    }
}

// EPI_STORE_ROWSTAT: softmax partials of one row over this wave's 32*TN columns (those < n_valid):
// (max, sum exp(C - max)) reduced over the row's two lanes (l, l ^ 32), stored as one float2 per
// (row, column group) at rowpart + 2 * (row * ld_rowpart + c0 / (32 * TN)).
template <int TM, int TN>
__device__ __forceinline__ void rowstat_slice(const GemmP &P, const f32x16 (&acc)[TM][TN], int i, int row, int c0,
                                              int kh) {
    float m = -INFINITY;
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
            for (int c = 0; c < 4; ++c)
                if (c0 + j * 32 + 8 * g + 4 * kh + c < P.n_valid) m = fmaxf(m, P.alpha * acc[i][j][4 * g + c]);
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    float l = 0.f;
    if (m != -INFINITY) {
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int g = 0; g < 4; ++g)
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    if (c0 + j * 32 + 8 * g + 4 * kh + c < P.n_valid) l += __expf(P.alpha * acc[i][j][4 * g + c] - m);
    }
    l += __shfl_xor(l, 32, 64);
    if (kh == 0)
        *reinterpret_cast<float2 *>(P.rowpart + 2 * ((int64_t)row * P.ld_rowpart + c0 / (32 * TN))) = make_float2(m, l);
}

// the epilogue operands of a 64 x 64 tile's (single) slice fetched before the main loop (pre_aux_epi)
template <int EPI>
constexpr int pre_aux_fetch = EPI == U2GNN_EPI_BIAS_DROP_RESID_LN ? U2GNN_EPI_BIAS_DROP_RESID : EPI;

template <int EPI, int TM, int TN>
__device__ __forceinline__ void store_tile(const GemmP &P, float *C, const f32x16 (&acc)[TM][TN], int r0, int c0,
                                           int li, int kh, const PreDS<TN> *pre,
                                           const EpiSlice<pre_aux_fetch<EPI>, TN> *pa = nullptr) {
    if constexpr (EPI == U2GNN_EPI_BIAS_DROP_RESID_LN) {
        store_tile_ln<TM, TN>(P, C, acc, r0, c0, li, kh, pa);
        return;
    }
    if constexpr (ds_signed<EPI>) {
        // every slice's probability image is requested before the first store (slice 0 usually
        // prefetched before the main loop): one exposed round trip per tile instead of one per slice
        EpiSlice<EPI, TN> e[TM];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            if (i == 0 && pre) slice_from_pre<EPI>(*pre, kh, e[i]);
            else fetch_slice<EPI>(P, r0 + i * 32 + li, c0, kh, e[i]);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i) store_slice<EPI>(P, C, acc, i, r0 + i * 32 + li, c0, kh, e[i]);
        return;
    }
    float rs[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int row = r0 + i * 32 + li;
        EpiSlice<EPI, TN> e;
        if constexpr (pre_aux_fetch<EPI> == EPI) {
            if (i == 0 && pa) {
                e = *pa;
                rs[i] = store_slice<EPI>(P, C, acc, i, row, c0, kh, e);
                continue;
            }
        }
        if (i == 0 && pre) slice_from_pre<EPI>(*pre, kh, e);
        else fetch_slice<EPI>(P, row, c0, kh, e);
        rs[i] = store_slice<EPI>(P, C, acc, i, row, c0, kh, e);
        if constexpr (EPI == U2GNN_EPI_STORE_ROWSTAT) rowstat_slice<TM, TN>(P, acc, i, row, c0, kh);
    }
    if constexpr (EPI == U2GNN_EPI_STORE_ROWDOT) {
        // one row partial per 64 output columns: lanes l and l + 32 hold a row's two column halves of
        // each MFMA tile; 64-column waves (TN == 2) own a group, 32-column waves (64 x 64 blocks of
        // 2 x 2 waves) add their neighbour's half through LDS
        static_assert(TN == 1 || TN == 2, "STORE_ROWDOT: 32- or 64-column wave tiles");
#pragma unroll
        for (int i = 0; i < TM; ++i) rs[i] += __shfl_xor(rs[i], 32, 64);
        if constexpr (TN == 2) {
#pragma unroll
            for (int i = 0; i < TM; ++i)
                if (kh == 0) P.rowpart[(int64_t)(c0 >> 6) * P.ld_rowpart + r0 + i * 32 + li] = rs[i];
        } else {
            static_assert(TM == 1, "STORE_ROWDOT: 64 x 64 blocks of 2 x 2 waves");
            __shared__ float rdred[64];
            const int row = r0 + li, rb = row & 63, wn = (c0 & 63) >> 5;
            if (kh == 0 && wn == 1) rdred[rb] = rs[0];
            __syncthreads();
            if (kh == 0 && wn == 0) P.rowpart[(int64_t)(c0 >> 6) * P.ld_rowpart + row] = rs[0] + rdred[rb];
        }
    }
}

// 1-D grid over gm * gn * split blocks.  The hardware deals workgroups to the 8 XCDs round-robin
// by linear id, so the bijective remap gives each XCD one contiguous range of logical ids; the
// logical order is split-slowest, then 8-row-tile groups with the row tile fastest inside a
// group.  Blocks that share an A row-panel or a B column-panel of the same K range therefore run
// on the same XCD (one L2), and the large N^2 operands of the skinny attention products are
// fetched from HBM once.
__device__ __forceinline__ int xcd_wgid() {
    const int bid = blockIdx.x;
    const int total = (int)gridDim.x;
    const int q = total >> 3, r = total & 7, xcd = bid & 7, loc = bid >> 3;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

// logical id -> (row tile, column tile, split) of a gm x gn grid
__device__ __forceinline__ void tile_of(int gm, int gn, int wgid, int &tm, int &tn, int &z) {
    const int ntile = gm * gn;
    z = wgid / ntile;
    const int t = wgid - z * ntile;
    constexpr int GROUP = 8;   // (16 and 13: C4 2.846 / 2.841 and 2.818 / 2.835 vs 2.808 / 2.811 ms, r05)
    const int per_group = GROUP * gn;
    const int g = t / per_group;
    const int first_m = g * GROUP;
    const int gsz = min(gm - first_m, GROUP);
    const int in_g = t - g * per_group;
    tm = first_m + in_g % gsz;
    tn = in_g / gsz;
}

__device__ __forceinline__ void tile_coords(int gm, int gn, int &tm, int &tn, int &z) {
    tile_of(gm, gn, xcd_wgid(), tm, tn, z);
}
}  // namespace
