/*
 * u2gnn_hip.h — C ABI of libu2gnn_hip.so, the MI355X (gfx950) kernels of the U2GNN hot path.
 *
 * The reference (shaginhekvs/Graph-Transformer, PyTorch) has no native kernels: every op
 * below replaces ATen calls made from the reference's Python.  Each entry point cites the
 * reference line whose computation it takes over (paths relative to the reference root).
 *
 * Conventions (all entry points):
 *   - plain pointers to DEVICE memory allocated by the caller; no allocation inside,
 *     no host synchronisation, so every call can be captured into a hipGraph;
 *   - `stream` is a hipStream_t passed as void* (NULL = the default stream);
 *   - fp32 row-major matrices with explicit leading dimensions (elements);
 *   - "padded" layouts: node rows padded to Np (multiple of 128), feature columns padded
 *     to a multiple of 64; padding columns are kept at zero by the producers;
 *   - return value: 0 on success, a negative U2GNN_E* code for argument errors, or a
 *     positive hipError_t from the launch.
 *   - dropout: keep(i,j) = hash(seed, i, j) >= p (counter-based; the same mask is
 *     regenerated in backward from (seed, i, j) — nothing is stored).
 */
#ifndef U2GNN_HIP_H
#define U2GNN_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define U2GNN_ABI_VERSION 18

#define U2GNN_OK 0
#define U2GNN_E_ARG (-1)    /* bad size / null pointer */
#define U2GNN_E_ALIGN (-2)  /* pointer or leading dimension not 16-byte aligned */
/* default tile rule (gemm args tile = 0): 256x128 blocks once a bf16x3/bf16 product has at least this
 * many of them (3 waves of 256 CUs); the shallow-K no-split path of the layer executor uses it too */
#define U2GNN_BIG_TILE_BLOCKS 768
#define U2GNN_E_SHAPE (-3)  /* dimension not a multiple of the kernel tile */

/* GEMM epilogues (u2gnn_gemm_args.epilogue). acc = sum_k A(m,k) B(k,n). */
#define U2GNN_EPI_STORE 0           /* C = alpha*acc                                     */
#define U2GNN_EPI_BIAS 1            /* C = (acc + bias[n]) * (n < scale_cols ? alpha : 1) */
#define U2GNN_EPI_BIAS_DROP_RESID 2 /* C = aux0[m,n] + drop(acc + bias[n])               */
#define U2GNN_EPI_BIAS_RELU_DROP 3  /* C = drop(relu(acc + bias[n]))                      */
#define U2GNN_EPI_RELU_DROP_BWD 4   /* C = acc * (aux0[m,n] > 0 ? 1/(1-p) : 0)            */
#define U2GNN_EPI_ACCUM 5           /* C = C + alpha*acc                                  */
#define U2GNN_EPI_ATTN_DS 6         /* C = aux1[m,n]*acc - aux0[m,n]*rowvec[m]; with keep:
                                       C = aux0[m,n]*(keep(m,n) ? acc/(1-p_drop) : 0 - rowvec[m]) */
#define U2GNN_EPI_ATTN_DS_SIGNED 7  /* aux0 = x, the signed probability image of
                                       u2gnn_attn_softmax_fwd (P == NULL): C = x*(acc - (1-p)*rowvec[m])
                                       where x >= +0 (kept), C = x*rowvec[m] where x <= -0 (dropped) */
#define U2GNN_EPI_ATTN_DS_RECOMP 8  /* retired in ABI v13 (it served the removed pre-split GEMM path):
                                       u2gnn_gemm returns U2GNN_E_ARG for it */
#define U2GNN_EPI_BIAS_DROP_RESID_LN 9 /* ABI v7: C = Z = aux0 + drop(acc + bias) as BIAS_DROP_RESID, and ln_y = the
                                          post-LayerNorm of Z's first ln_d columns (ln_gamma, ln_beta, ln_eps;
                                          ln_mean / ln_rstd per row; rows >= ln_rows and columns >= ln_d
                                          written as 0).  Row-complete tiles only: N == 64 (tile 64),
                                          bf16 / bf16x3, split_k 1 -- the d <= 64 encoders (C3, C5) */
#define U2GNN_EPI_STORE_ROWDOT 10   /* ABI v8: C = alpha*acc as STORE, and per 64-column group q = n/64 the
                                       row partial rowpart[q*ld_rowpart + m] = sum_{n in q} C[m,n]*aux0[m,n]
                                       (the attention backward's delta = rowsum(dO * O) formed by the dO
                                       GEMM; ATTN_DS_SIGNED sums the N/64 partials in q order, rowvec_parts).
                                       N % 64 == 0, split_k 1, fp32-operand kernels only */
#define U2GNN_EPI_STORE_ROWSTAT 11 /* ABI v10: C = alpha*acc as STORE, and per row m and group q of 32*TN
                                       output columns (the wave tile's width: 64 on 128- and 256-row tiles, 32 on
                                       64x64 tiles) the softmax partials over the columns n < n_valid (columns
                                       n >= n_valid are stored as -inf: masked keys): rowpart[2*(m*ld_rowpart + q)] = max, [+1] =
                                       sum exp(C - max) (-inf and 0 when the group has no such column) -- the
                                       attention scores S = Q K^T and their row statistics in one pass
                                       (u2gnn_attn_softmax_pv folds the groups).  bf16 kinds, split_k 1 */

/* x2 operand format (pre-split fp32): a logical fp32 matrix X[R][C] (C % 8 == 0) is stored as
 * bf16 X2[R][2C] with, per 8-column group g, hi(X[r][8g..8g+7]) then lo(X[r][8g..8g+7]),
 * hi = bf16_rne(x), lo = bf16_rne(x - hi).  Leading dimensions of x2 matrices are in bf16
 * elements (>= 2C, multiple of 16).  The bf16x3 product hi*hi + hi*lo + lo*hi of two x2 operands
 * is the one the BF16X3 kernels form after splitting fp32 operands themselves, so an x2 GEMM
 * is bit-identical to the fp32-operand BF16X3 GEMM on the same 256x128 / 128x128 tile. */

/* Matrix-core precision of a GEMM (u2gnn_gemm_args.precision). */
#define U2GNN_PREC_F32 0    /* v_mfma_f32_32x32x2_f32: exact fp32 fma chains            */
#define U2GNN_PREC_BF16X3 1 /* split-bf16 (hi*hi+hi*lo+lo*hi) on bf16 MFMA, fp32 accum  */
#define U2GNN_PREC_BF16 2   /* plain bf16 operands on bf16 MFMA, fp32 accum             */
#define U2GNN_PREC_BF16X6 3 /* ABI v17: three-way split x = hi + mid + lo (bf16 each, exact for fp32 x);
                               hh + hm + mh + hl + lh + mm on bf16 MFMA, fp32 accum (~2^-26 per product,
                               the fp32 products' accuracy at 6/16 of the bf16 rate).  16-deep K step on
                               every tile; A not transposed (the forward products' layouts) */
#define U2GNN_PREC_F16X3 4  /* ABI v18: two-way fp16 split x = hi + lo, hi = fp16_rne(x), lo = fp16_rne(x - hi)
                               (11 + 11 significant bits), hh + hl + lh on fp16 MFMA, fp32 accum (~2^-21 per
                               product at the bf16x3 rate).  |x| < 65504 (hi overflows to inf beyond); x small
                               enough that lo is subnormal keeps an absolute error <= 2^-25.  The forward
                               products' epilogues and layouts, as U2GNN_PREC_BF16X6 */

typedef struct u2gnn_gemm_args {
    const float *A;       /* trans_a=0: A[m*lda+k]   trans_a=1: A[k*lda+m] */
    const float *B;       /* trans_b=0: B[k*ldb+n]   trans_b=1: B[n*ldb+k] */
    float *C;             /* C[m*ldc+n]; with split_k>1: slab z at C + z*slab_stride */
    int64_t M, N, K;
    int64_t lda, ldb, ldc;
    int32_t trans_a, trans_b;
    int32_t epilogue;     /* U2GNN_EPI_*; split_k>1 requires STORE */
    int32_t split_k;      /* >= 1; K (a multiple of the K tile: 16 fp32, 32 bf16 modes) is cut into
                             split_k chunks of Kc = ceil(K/(split_k*tile))*tile; slab z holds the
                             partial sum over [z*Kc, min((z+1)*Kc, K)) (zeros when empty) */
    int64_t slab_stride;
    const float *bias;    /* [N] */
    const float *aux0;    /* residual / saved relu-dropout output / P */
    const float *aux1;    /* Pd (dropped probabilities) */
    const float *rowvec;  /* [M] (delta of the attention backward) */
    int64_t ld_aux;
    float alpha;
    int64_t scale_cols;
    float p_drop;
    uint64_t seed;
    int32_t precision;    /* U2GNN_PREC_* */
    int32_t tile;         /* 0 = auto; 64 / 128 square block tiles; bf16 modes also 256 (256x128
                             block, 8 waves) and 129 (128x128 block with a 16-deep K step, 3
                             blocks per CU: skinny weight-gradient products) */
    const uint32_t *keep; /* ATTN_DS: dropout keep bits of the probabilities (bit n%32 of
                             keep[m*ld_keep + n/32]) written by u2gnn_attn_softmax_fwd, or NULL
                             (then aux1 = Pd is read) */
    int64_t ld_keep;      /* words per row of keep */
    int32_t clamp_a;      /* 1: A elements below +0 are read as 0 (the signed probability image as Pd
                             for P.V and dP^T.dO); STORE epilogue and trans_b = 0 only */
    int32_t cx2_col0;     /* ABI v12: Cx2 receives only output columns >= cx2_col0 (a multiple of 8; 0 = all):
                             the in-projection writes the x2 copy of its V block only */
    /* ---- ABI v3: pre-split (x2) operands and outputs ---- */
    int32_t a_x2, b_x2;   /* retired: the pre-split operand kernels were removed in round 4; must be 0
                             (else U2GNN_E_ARG).  The fields keep the struct layout. */
    const void *A2;       /* unused (retired with a_x2 / b_x2) */
    const void *B2;
    void *Cx2;            /* non-NULL: the epilogue result is also (C == NULL: only) written in x2
                             format, ldcx2 bf16 elements per row; split_k must be 1; not with
                             ATTN_DS_SIGNED, whose result goes to C only (round 5) */
    int64_t ldcx2;
    const float *rowstat; /* unused since ABI v13 (the retired ATTN_DS_RECOMP epilogue); layout kept */
    int64_t m_valid, n_valid;   /* m_valid unused since v13; n_valid: STORE_ROWSTAT's real keys (columns) */
    /* ---- ABI v7: LayerNorm fused into the bias-dropout-residual epilogue (EPI_BIAS_DROP_RESID_LN) ---- */
    const float *ln_gamma, *ln_beta;   /* [ln_d], any 4-byte alignment */
    float *ln_y;                       /* [M][ln_ldy], 16-byte aligned rows */
    int64_t ln_ldy;
    float *ln_mean, *ln_rstd;          /* [M] */
    int64_t ln_d, ln_rows;
    float ln_eps;
    int32_t ln_reserved;
    /* ---- ABI v8: delta from the dO GEMM (EPI_STORE_ROWDOT -> EPI_ATTN_DS_SIGNED) ---- */
    float *rowpart;       /* STORE_ROWDOT: [N/64][ld_rowpart] row partials (ld_rowpart >= M);
                             STORE_ROWSTAT (ABI v10): [M][ld_rowpart] (max, sum) float2 pairs, ld_rowpart in
                             pairs (>= N/32), 8-byte aligned; n_valid = the columns taken */
    int64_t ld_rowpart;
    int32_t rowvec_parts; /* ATTN_DS_SIGNED: 0/1 = rowvec[m]; P > 1 = sum_{q<P} rowvec[q*ld_rowvec + m] in
                             q order (fp32-operand kernels only) */
    int32_t rowvec_reserved;
    int64_t ld_rowvec;
    /* ---- ABI v18: U2GNN_PREC_F16X3 operand pre-scales ---- */
    int32_t h3_exp_a, h3_exp_b;   /* A and B are multiplied by 2^h3_exp_a / 2^h3_exp_b before the fp16 split and the
                                     result by 2^-(h3_exp_a + h3_exp_b) before the epilogue (exact): a scale that
                                     puts an operand's typical magnitude near 2^3 keeps lo normal (22 bits) for
                                     elements down to 2^-9 of it (the layer executor: 6 for activations and
                                     weights, 15 - ceil(log2(1/(1-p))) for the probability image, whose entries
                                     are ~1/N).  Within [-24, 24]; must be 0 for the other precisions */
} u2gnn_gemm_args;

/* ---- library ------------------------------------------------------------------ */
int u2gnn_abi_version(void);

/* ---- a2: neighbour gather  (pytorch_U2GNN_Sup.py:32,39; pytorch_U2GNN_UnSup.py:54) --------
 * dst[i, 0:d] = src[idx[i*idx_stride], 0:d] for i < n_rows; dst[i, d:d_pad] = 0;
 * rows n_rows..n_rows_pad-1 = 0.  Out-of-range indices write zeros and set *err = 1. */
int u2gnn_gather_rows(const float *src, int64_t ld_src, int64_t src_rows, const int64_t *idx,
                      int64_t idx_stride, float *dst, int64_t ld_dst, int64_t n_rows,
                      int64_t n_rows_pad, int64_t d, int64_t d_pad, int32_t *err, void *stream);
/* backward of the gather: dst[idx[i*idx_stride], 0:d] += src[i, 0:d] (fp32 atomics) for i < n_rows.
 * Indices outside [0, dst_rows) add nothing and set *err = 1 (err may be NULL). */
int u2gnn_scatter_add_rows(const float *src, int64_t ld_src, const int64_t *idx, int64_t idx_stride,
                           float *dst, int64_t ld_dst, int64_t dst_rows, int64_t n_rows, int64_t d,
                           int32_t *err, void *stream);

/* ---- a3.x: every dense contraction of the encoder (in-proj, Q.K^T, P.V, out-proj, FFN)
 * and of its backward  (torch TransformerEncoderLayer at pytorch_U2GNN_Sup.py:19-21,35;
 * pytorch_U2GNN_UnSup.py:37-40,57) -------------------------------------------------- */
int u2gnn_gemm(const u2gnn_gemm_args *args, void *stream);

/* split-K / padded -> real unpack:  dst[map(r), map(c)] (+)= alpha * sum_z src[z*slab_stride + r*ld_src + c]
 * for r < rows_pad, c < cols_pad whose in-block index is < the real block size; the map
 * packs blocks of size (blk_pad) to (blk_real): r -> (r / rblk_pad) * rblk_real + r % rblk_pad. */
int u2gnn_slab_reduce(const float *src, int32_t n_slab, int64_t slab_stride, int64_t rows_pad,
                      int64_t cols_pad, int64_t ld_src, int64_t rblk_pad, int64_t rblk_real,
                      int64_t cblk_pad, int64_t cblk_real, float *dst, int64_t ld_dst, float alpha,
                      int32_t accumulate, void *stream);

/* pack real-shaped parameters into padded device buffers (same block map as above, inverse);
 * padding entries of dst are written with 0. */
int u2gnn_pack_padded(const float *src, int64_t ld_src, int64_t rows_pad, int64_t cols_pad,
                      int64_t rblk_pad, int64_t rblk_real, int64_t cblk_pad, int64_t cblk_real,
                      float *dst, int64_t ld_dst, void *stream);

/* many u2gnn_pack_padded jobs in one launch (the descriptor array is a HOST array; up to 32 jobs
 * per launch, more are split into several launches). */
typedef struct u2gnn_pack_desc {
    const float *src;
    float *dst;
    int64_t ld_src, rows_pad, cols_pad, rblk_pad, rblk_real, cblk_pad, cblk_real, ld_dst;
} u2gnn_pack_desc;
int u2gnn_pack_padded_multi(const u2gnn_pack_desc *descs, int32_t n, void *stream);
/* ABI v11: the same, and the launch also performs u2gnn_step_advance(epoch, t) (either may be NULL) before any
 * later launch on the stream runs: the first node of a replayed step without a launch of its own (n >= 1). */
int u2gnn_pack_padded_multi_adv(const u2gnn_pack_desc *descs, int32_t n, uint64_t *epoch, int64_t *t,
                                void *stream);

/* column sums (bias gradients):  out[map(c)] (+)= sum_{r<rows} X[r*ld + c], c < cols_pad.
 * ws must hold ceil(rows/16) * cols_pad floats (kernels.colstat_ws_floats allocates 3x that); 16-byte
 * loads when X, ws are 16-byte aligned with ld and cols_pad multiples of 4, scalar loads otherwise. */
int u2gnn_colsum(const float *X, int64_t rows, int64_t cols_pad, int64_t ld, int64_t cblk_pad,
                 int64_t cblk_real, float *out, int32_t accumulate, float *ws, void *stream);

/* ---- a3.2: attention row softmax + dropout(p) on probabilities (MHA core) ----------
 * P[i,j] = softmax_j(S[i,j], j < n_valid); Pd = P * keep / (1-p); rows >= rows_valid -> 0.
 * Pd may alias P when p == 0.  P == NULL selects the signed image: Pd = P/(1-p) where kept and
 * -P where dropped (the sign bit carries the keep decision; keep must then be NULL), consumed by
 * the clamp_a GEMMs and U2GNN_EPI_ATTN_DS_SIGNED.  keep (optional, n_pad % 32 == 0): the keep decisions as bits,
 * bit j%32 of keep[i*ld_keep + j/32] (0 for j >= n_valid and padded rows), for the ATTN_DS
 * epilogue of the backward.  Rows are held in registers: n_pad <= 32768 (else U2GNN_E_SHAPE). */
int u2gnn_attn_softmax_fwd(const float *S, int64_t lds, float *P, float *Pd, int64_t ldp,
                           int64_t rows_valid, int64_t rows_pad, int64_t n_valid, int64_t n_pad,
                           float p, uint64_t seed, uint32_t *keep, int64_t ld_keep, void *stream);
/* delta[i] = sum_c A[i,c]*B[i,c]  (rowsum(dO * O) of the attention backward) */
/* dst2 = x2(src) over rows x cols (cols % 8 == 0; ld_dst2 in bf16 elements) */
int u2gnn_split_x2(const float *src, int64_t ld_src, void *dst2, int64_t ld_dst2, int64_t rows, int64_t cols,
                   void *stream);
int u2gnn_rowdot(const float *A, int64_t lda, const float *B, int64_t ldb, float *out, int64_t rows,
                 int64_t cols, void *stream);

/* ---- a3.3 / a3.4: post-LN  (norm1/norm2, eps 1e-5) -------------------------------------
 * Y = LN(Z) over the first d columns; Y[:, d:d_pad] = 0; rows >= rows_valid -> 0. */
int u2gnn_layernorm_fwd(const float *Z, int64_t ldz, const float *gamma, const float *beta, float *Y,
                        int64_t ldy, float *mean, float *rstd, int64_t rows_valid, int64_t rows_pad,
                        int64_t d, int64_t d_pad, float eps, void *stream);
/* dZ = LN'(dY) (rows >= rows_valid and columns >= d written 0); dZdrop = dZ * keep/(1-p)
 * (may be NULL): the gradient of the dropout branch that fed this LN's residual sum. */
int u2gnn_layernorm_bwd(const float *dY, int64_t ldy, const float *Z, int64_t ldz, const float *mean,
                        const float *rstd, const float *gamma, float *dZ, int64_t lddz, float *dZdrop,
                        int64_t lddrop, float p, uint64_t seed, int64_t rows_valid, int64_t rows_pad,
                        int64_t d, int64_t d_pad, void *stream);
/* ABI v8: u2gnn_layernorm_bwd of an encoder layer's LayerNorm1 that also writes the attention backward's
 * delta[r] = sum_{c<d_pad} dZdrop[r,c] * ((Z - X)[r,c] * (1-p) - bias[c]) (0 for r >= rows_valid), where
 * Z = X + drop(O W_o^T + bias) is the LN input, X the layer input and bias the zero-padded out-projection
 * bias: in exact arithmetic rowsum(dO * O) with dO = dZdrop W_o (u2gnn_rowdot), without reading dO or O.
 * X [rows_pad][ldx] and bias [d_pad] 16-byte aligned; delta [rows_pad]. */
int u2gnn_layernorm_bwd_delta(const float *dY, int64_t ldy, const float *Z, int64_t ldz, const float *mean,
                              const float *rstd, const float *gamma, float *dZ, int64_t lddz, float *dZdrop,
                              int64_t lddrop, float p, uint64_t seed, int64_t rows_valid, int64_t rows_pad,
                              int64_t d, int64_t d_pad, const float *X, int64_t ldx, const float *bias,
                              float *delta, void *stream);
/* ABI v11: u2gnn_layernorm_bwd_delta whose dY is first completed by split-K slabs: dY[r, c] += sum_z
 * slabs[z*slab_stride + r*ldy + c] (u2gnn_slab_reduce's summation order, accumulate; written back to dY for
 * rows < rows_valid) -- the FFN's dX1 += dH W1 product of a one-stream layer without its reduce launch. */
int u2gnn_layernorm_bwd_delta_slabs(float *dY, int64_t ldy, const float *slabs, int32_t n_slab, int64_t slab_stride,
                                    const float *Z, int64_t ldz, const float *mean, const float *rstd,
                                    const float *gamma, float *dZ, int64_t lddz, float *dZdrop, int64_t lddrop, float p,
                                    uint64_t seed, int64_t rows_valid, int64_t rows_pad, int64_t d, int64_t d_pad,
                                    const float *X, int64_t ldx, const float *bias, float *delta, void *stream);
/* LN parameter gradients: dgamma[c] = sum_r dY*xhat, dbeta[c] = sum_r dY (c < d) and, when
 * dbias != NULL, dbias[c] = sum_r dZdrop[r, c] (bias of the linear whose output was dropped into
 * the residual: out_proj.bias for norm1, linear2.bias for norm2).  Deterministic two-pass column
 * reduction; ws >= ceil(rows_valid/16) * 3 * d_pad floats; dY, Z, dZdrop, ws 16-byte aligned with
 * leading dimensions and d_pad multiples of 4. */
int u2gnn_layernorm_bwd_params(const float *dY, int64_t ldy, const float *Z, int64_t ldz,
                               const float *mean, const float *rstd, const float *dZdrop,
                               int64_t lddrop, int64_t rows_valid, int64_t d, int64_t d_pad, float *ws,
                               float *dgamma, float *dbeta, float *dbias, void *stream);

/* ---- ABI v11: batched reductions -------------------------------------------------------------
 * Many u2gnn_slab_reduce / u2gnn_colsum / u2gnn_layernorm_bwd_params jobs in at most two launches (the
 * column partials of every long job, then every combine; jobs over <= 512 rows take the one-launch small
 * forms), each job with the per-element arithmetic and summation order of its single-job call, so the
 * results are bit-identical.  Jobs must write distinct outputs.  Fields per kind:
 *   SLAB:     src, n_slab, slab_stride, rows (= rows_pad), cols (= cols_pad), ld_src, rblk_*, cblk_*,
 *             dst, ld_dst, alpha, accumulate                       (u2gnn_slab_reduce)
 *   COLSUM:   src (= X), rows, cols (= cols_pad), ld_src, cblk_*, dst, accumulate   (u2gnn_colsum)
 *   LNPARAMS: src (= dY), ld_src, Z, ldz, mean, rstd, dZdrop, lddrop, rows (= rows_valid), d,
 *             cols (= d_pad), dst (= dgamma), dbeta, dbias      (u2gnn_layernorm_bwd_params)
 * COLSUM / LNPARAMS need 16-byte aligned operands (leading dimensions and cols multiples of 4).
 * ws: >= u2gnn_reduce_batch_ws_floats(jobs, n) floats, 16-byte aligned (the partial sums). */
#define U2GNN_RJOB_SLAB 0
#define U2GNN_RJOB_COLSUM 1
#define U2GNN_RJOB_LNPARAMS 2
typedef struct u2gnn_reduce_job {
    int32_t kind, n_slab, accumulate;
    float alpha;
    const float *src;
    int64_t ld_src, slab_stride, rows, cols, d;
    int64_t rblk_pad, rblk_real, cblk_pad, cblk_real;
    float *dst;
    int64_t ld_dst;
    const float *Z, *mean, *rstd, *dZdrop;
    int64_t ldz, lddrop;
    float *dbeta, *dbias;
} u2gnn_reduce_job;
int64_t u2gnn_reduce_batch_ws_floats(const u2gnn_reduce_job *jobs, int32_t n);
int u2gnn_reduce_batch(const u2gnn_reduce_job *jobs, int32_t n, float *ws, int64_t ws_floats, void *stream);

/* ABI v11: FFN2's epilogue when the product runs split-K (too few output tiles to fill the chip):
 * Z = resid + drop(sum_z src[z] + bias) (dropout hash of U2GNN_EPI_BIAS_DROP_RESID), then the LayerNorm of
 * EPI_BIAS_DROP_RESID_LN over the first d columns: Y, mean, rstd (rows >= rows_valid: 0).  d <= 256 (round 5;
 * d <= 64 before), padded width dp = rup(d, 64), one wave per row; bias / resid / slabs / Z / Y padded to dp
 * columns, gamma / beta unpadded [d].  For d <= 64 the results are the round-4 kernel's, bit for bit. */
int u2gnn_slab_bias_drop_resid_ln(const float *src, int32_t n_slab, int64_t slab_stride, int64_t ld_src,
                                   const float *bias, const float *resid, int64_t ld_res, float p, uint64_t seed,
                                   float *Z, int64_t ldz, const float *gamma, const float *beta, float *Y, int64_t ldy,
                                   float *mean, float *rstd, int64_t d, int64_t rows_valid, int64_t rows_pad, float eps,
                                   void *stream);

/* ABI v11: several u2gnn_gemm calls in one launch when they resolve to one grouped kernel: the same
 * bf16 precision and tile (64, 129 or 256), STORE epilogue (split-K allowed), B not transposed, each job
 * A^T B, A^T B with clamp_a, or A B.  The blocks of the launch are shared out over the jobs, each tile
 * computed exactly as by its own u2gnn_gemm call (bit-identical).  Otherwise the calls are launched one by
 * one.  At most 8 jobs. */
int u2gnn_gemm_group(const u2gnn_gemm_args *args, int32_t n, void *stream);

/* ---- ABI v11: UnSup head glue (pytorch_U2GNN_UnSup.py:52-69; the TF model's dropout before the sampled
 * softmax, U2GNN_tf/model_U2GNN_Unsup_multi.py:43-56) ---------------------------------------------------
 * u2gnn_concat_dropout: Y[r, l*d + c] = drop(src[l][r*ld_src + c]) for r < N, c < d, l < L (L <= 8; src a
 * HOST array of L device pointers; the mask of u2gnn_dropout(Y) over Y's indices; p = 0: a copy).
 * u2gnn_split_dropout_bwd: dst[l][r*dp + c] = drop(dY[r, l*d + c]) (same mask) for r < N, c < d, and 0 on
 * the padding (r < Np, c < dp): the layers' padded input gradients.
 * u2gnn_sum: out[0] = sum of x[0, n) in a fixed order (one block).
 * u2gnn_index_zero_rows2: u2gnn_index_zero_rows over two index sets in one launch (the sets may overlap). */
int u2gnn_concat_dropout(const float *const *src, int32_t L, int64_t ld_src, int64_t N, int64_t d, float p,
                         uint64_t seed, float *Y, int64_t ldy, void *stream);
int u2gnn_split_dropout_bwd(const float *dY, int64_t ldy, int32_t L, int64_t N, int64_t Np, int64_t d, int64_t dp,
                            float p, uint64_t seed, float *const *dst, void *stream);
int u2gnn_sum(const float *x, int64_t n, float *out, void *stream);
int u2gnn_index_zero_rows2(const int64_t *idx_a, int64_t n_a, const int64_t *idx_b, int64_t n_b, float *dst,
                           int64_t ld_dst, int64_t dst_rows, int64_t D, int32_t *err, void *stream);

/* ---- a5/a6: sum pooling + dropout + per-layer head  (pytorch_U2GNN_Sup.py:41-44) ------
 * G[b, c] = drop(sum_{e in [rowptr[b], rowptr[b+1])} vals[e] * X[colidx[e], c]), c < d;
 * G[b, d:ldg] untouched. */
int u2gnn_pool_fwd(const float *X, int64_t ldx, const int64_t *rowptr, const int64_t *colidx,
                   const float *vals, float *G, int64_t ldg, int64_t B, int64_t d, float p,
                   uint64_t seed, void *stream);
/* dX[colidx[e], c] += vals[e] * dGd[b, c] * keep/(1-p)   (fp32 atomics) */
int u2gnn_pool_bwd(const float *dGd, int64_t ldg, const int64_t *rowptr, const int64_t *colidx,
                   const float *vals, float *dX, int64_t ldx, int64_t B, int64_t d, float p,
                   uint64_t seed, void *stream);
/* ABI v8: pool backward for block-row pools, whose colidx[0, N) (N = rowptr[B]) holds every row index
 * 0..N-1 once: dX[colidx[e], c] = vals[e] * dGd[b, c] * keep/(1-p) for c < d, 0 for d <= c < d_pad,
 * and rows N..rows_pad-1 = 0 -- plain stores, so dX needs no zero fill (u2gnn_pool_bwd accumulates). */
int u2gnn_pool_bwd_rows(const float *dGd, int64_t ldg, const int64_t *rowptr, const int64_t *colidx,
                        const float *vals, float *dX, int64_t ldx, int64_t B, int64_t d, int64_t d_pad,
                        int64_t N, int64_t rows_pad, float p, uint64_t seed, void *stream);
/* scores[b, c] (+)= sum_j G[b, j] W[c, j] + bias[c]   (W real [C, d]) */
int u2gnn_head_fwd(const float *G, int64_t ldg, const float *W, const float *bias, float *scores,
                   int64_t B, int64_t C, int64_t d, int32_t accumulate, void *stream);
/* dG[b, j] = sum_c dS[b,c] W[c,j];  dW[c,j] (+)= sum_b dS[b,c] G[b,j];  db[c] (+)= sum_b dS[b,c] */
int u2gnn_head_bwd(const float *dscores, const float *G, int64_t ldg, const float *W, float *dG,
                   int64_t lddg, float *dW, float *db, int64_t B, int64_t C, int64_t d,
                   int32_t accumulate, void *stream);

/* ---- a7: label smoothing + soft cross-entropy  (pytorch_U2GNN_Sup.py:48-60;
 * train_pytorch_U2GNN_Sup.py:140-142,158) -----------------------------------------------
 * loss[0] = mean_b sum_c -t_bc log_softmax(s_b)_c ; dscores = (softmax - t) / B */
int u2gnn_smoothed_ce(const float *scores, const int64_t *labels, int64_t B, int64_t C,
                      float smoothing, float *loss, float *dscores, void *stream);

/* ---- a9: clip_grad_norm_(max_norm) + Adam  (train_pytorch_U2GNN_Sup.py:145,160-161) ----
 * sqnorm[0] = sum g^2 (double accumulation, fp32 result); ws >= 1024 floats. */
int u2gnn_sqnorm(const float *g, int64_t n, float *ws, float *sqnorm, void *stream);
/* ABI v11: the clip + Adam pair in two launches instead of three: u2gnn_sqnorm_partials writes the per-block
 * partial sums of g^2 into ws (>= 1024 floats); u2gnn_adam_sq / u2gnn_adam_dev_sq (the arguments of
 * u2gnn_adam / u2gnn_adam_dev with ws in place of sqnorm) fold them in every block in u2gnn_sqnorm's order
 * (the same clip coefficient, bit for bit) and store the total into sqnorm (may be NULL). */
int u2gnn_sqnorm_partials(const float *g, int64_t n, float *ws, void *stream);
int u2gnn_adam_sq(float *param, const float *grad, float *exp_avg, float *exp_avg_sq, int64_t n, const float *ws,
                  float *sqnorm, float max_norm, float beta1, float beta2, float eps, float step_size, float bc2_sqrt,
                  void *stream);
int u2gnn_adam_dev_sq(float *param, const float *grad, float *exp_avg, float *exp_avg_sq, int64_t n, const float *ws,
                      float *sqnorm, float max_norm, double beta1, double beta2, float eps, const double *lr,
                      const int64_t *step, void *stream);
/* torch.optim.Adam single-tensor step on a flat buffer with the clip coefficient
 * min(1, max_norm/(sqrt(*sqnorm)+1e-6)) applied to g on the fly (sqnorm NULL: no clip).
 * step_size = lr / (1 - beta1^t), bc2_sqrt = sqrt(1 - beta2^t), computed by the caller. */
int u2gnn_adam(float *param, const float *grad, float *exp_avg, float *exp_avg_sq, int64_t n,
               const float *sqnorm, float max_norm, float beta1, float beta2, float eps,
               float step_size, float bc2_sqrt, void *stream);

/* ---- a10: sampled softmax  (sampled_softmax.py:36-56) --------------------------------------
 * loss_i = log sum_s exp(x_i . w_s) - x_i . w_{y_i}   (== the reference -log(exp(t)/sum exp(s))
 * whenever the reference is finite); prob[i, s] = softmax over samples (saved for backward). */
int u2gnn_sampled_softmax_fwd(const float *X, int64_t ldx, const int64_t *labels,
                              const int64_t *sample_ids, int64_t S, const float *W, int64_t ldw,
                              float *loss, float *prob, int64_t n_rows, int64_t D, void *stream);
/* with upstream dloss[i] (NULL = all ones): dX[i] = dloss_i (sum_s prob_is w_s - w_{y_i});
 * dW[y_i] -= dloss_i x_i;  dW[s] += sum_i dloss_i prob_is x_i   (dW accumulated, atomics) */
int u2gnn_sampled_softmax_bwd(const float *X, int64_t ldx, const int64_t *labels,
                              const int64_t *sample_ids, int64_t S, const float *W, int64_t ldw,
                              const float *prob, const float *dloss, float *dX, int64_t lddx,
                              float *dW, int64_t lddw, int64_t n_rows, int64_t D, void *stream);
/* ABI v9: the same backward with W's gradient as compact rows instead of a dense [V, D] image:
 * dW_lab[i] = -dloss_i x_i  (row of W labels[i]),  dW_smp[j] = sum_i dloss_i prob_ij x_i  (row of W
 * sample_ids[j]).  Plain stores, no atomics, no zero fill: the rows are what the data-parallel
 * exchange all-gathers (train_pytorch_U2GNN_UnSup.py:149-162, sampled_softmax.py:45,48 touch only
 * these rows), and u2gnn_index_add_rows folds them into the dense gradient. */
int u2gnn_sampled_softmax_bwd_rows(const float *X, int64_t ldx, const int64_t *labels,
                                   const int64_t *sample_ids, int64_t S, const float *W, int64_t ldw,
                                   const float *prob, const float *dloss, float *dX, int64_t lddx,
                                   float *dW_lab, int64_t ld_lab, float *dW_smp, int64_t ld_smp, int64_t n_rows,
                                   int64_t D, void *stream);

/* ---- ABI v9: row-indexed updates of a dense [V, D] buffer ------------------------------------
 * dst[idx[r], c] += alpha * src[r, c] (r < n_rows, c < D).  The idx entries of ONE call must be
 * distinct (plain read-modify-write, no atomics): callers order overlapping sets over separate calls,
 * which makes the sum order, and so the bits, fixed.  idx outside [0, dst_rows) is skipped and sets
 * *err (when err is non-NULL). */
int u2gnn_index_add_rows(const float *src, int64_t ld_src, const int64_t *idx, int64_t n_rows, float alpha,
                         float *dst, int64_t ld_dst, int64_t dst_rows, int64_t D, int32_t *err, void *stream);
/* dst[idx[r], c] = 0 for r < n_rows, c < D (duplicates allowed); out-of-range idx skipped + *err. */
int u2gnn_index_zero_rows(const int64_t *idx, int64_t n_rows, float *dst, int64_t ld_dst, int64_t dst_rows,
                          int64_t D, int32_t *err, void *stream);

/* ---- ABI v10: fused softmax -> dropout -> P.V over the node axis (a3.2; pytorch_U2GNN_Sup.py:19-21,35) ----
 * The attention forward after S = Q K^T (u2gnn_gemm with EPI_STORE_ROWSTAT, whose epilogue leaves per row
 * the (max, sum exp) partials of ngroups column groups in rowpart, ld_rowpart pairs per row): the
 * probabilities never exist apart from the one signed image the backward reads.  Per row m < n_valid the
 * kernel folds the partials into (M, L) and, for keys n < n_valid, P = exp(S[m,n] - M) / L, keep =
 * keep(seed, m, n) (the hash of every dropout site); it writes the signed image Pd = keep ? P/(1-p) : -P
 * (zero for padded rows / keys; what EPI_ATTN_DS_SIGNED and the clamped P^T.dO read) and
 * O = Pd_kept . V on the matrix cores (precision BF16X3: split-bf16, 3 products; BF16: 1), V read from qkv2
 * (the in-projection output in x2 format, [rows_pad][ldq2] bf16, V = columns 2dp .. 3dp).  ABI v17, precision
 * BF16X6: qkv2 is the fp32 in-projection output itself ([rows_pad][ldq2] float, ldq2 >= 3 dp, V = columns
 * 2dp .. 3dp), P and V split three ways in registers, 6 products (fp32-accurate).  ABI v18, precision F16X3:
 * qkv2 in x2 layout holding fp16 planes of 2^U2GNN_H3_X2_EXP times the in-projection output (what an F16X3 GEMM
 * writes to Cx2), P scaled by 2^(15 - ceil(log2(1/(1-p)))) and split into fp16 hi / lo, 3 fp16 products, O
 * scaled back (f16x3 accuracy).  dp in {64, 128,
 * ..., 384}, rows_pad % 128 == 0, ngroups and ld_rowpart even, rowpart 16-byte aligned; S columns >= n_valid
 * hold -inf (as EPI_STORE_ROWSTAT writes them); S and Pd may alias (the image is written over the scores).
 * ws: u2gnn_attn_softmax_pv_ws_floats(n_valid, rows_pad, dp) floats (per key range partial outputs). */
int64_t u2gnn_attn_softmax_pv_ws_floats(int64_t n_valid, int64_t rows_pad, int64_t dp);
int u2gnn_attn_softmax_pv(const float *S, int64_t lds, const float *rowpart, int64_t ld_rowpart, int64_t ngroups,
                          const void *qkv2, int64_t ldq2, int64_t dp, float *Pd, int64_t ldp, float *O, int64_t ldo,
                          float *ws, int64_t ws_floats, int64_t n_valid, int64_t rows_pad, float p, uint64_t seed,
                          int32_t precision, void *stream);

/* ---- ABI v15: in-projection + node-axis attention for small widths d <= 32 (a3.1 + a3.2 forward and backward;
 * the UnSup encoders) -- exact fp32 on the vector ALUs, flash-style: no N x N image and no [rows_pad][3 dp] QKV
 * image are stored.  Keys / queries n < n_valid take part, keep = keep(seed, m, n) as every dropout site.
 * fwd: (Q, K, V) = X W_in^T + b_in with Q scaled by 1/sqrt(d) (X [rows_pad][ldx], d real columns, the rest zero;
 *      W_in [3 dp][dp] and b_in [3 dp] in the executor's padded layout, dp = 64), then O[m] = sum_n keep P[m,n] /
 *      (1-p) V[n] with P = softmax_n(Q[m].K[n]) (rows >= n_valid and columns >= d written 0), and the forward
 *      context ctx (u2gnn_attn_small_ctx_floats(rows_pad, d) floats, 16-byte aligned): ctx[2m], ctx[2m+1] =
 *      (max_n Q[m].K[n] log2 e, 1 / sum_n exp) -- what the backward recomputes P from -- followed by a compact
 *      copy of Q, K, V (rows >= n_valid zero).
 * bwd: given the forward's ctx (unchanged), dO and delta[m] = rowsum(dO[m] * O[m]): dQKV (all 3 dp columns of
 *      every row written; padding 0) = (q_scale * dS K, dS^T Q, Pd^T dO) with dS = P o (keep dO.V^T / (1-p) -
 *      delta), Pd = keep P / (1-p) -- the gradients of the in-projection's (pre-scale) outputs -- and, unless dX
 *      is NULL, dX[m] += dQKV[m] W_in (the in-projection's input gradient, rows < n_valid, columns < d).
 *      ws: u2gnn_attn_small_ws_floats(n_valid, rows_pad, d) floats of scratch (per-query records), 16-byte
 *      aligned.  Both sizing functions return -1 for d > 32 (the matrix-core path's widths). */
int64_t u2gnn_attn_small_ctx_floats(int64_t rows_pad, int64_t d);
int64_t u2gnn_attn_small_ws_floats(int64_t n_valid, int64_t rows_pad, int64_t d);
int u2gnn_attn_small_fwd(const float *X, int64_t ldx, const float *W_in, const float *b_in, int64_t dp, int64_t d,
                         int64_t n_valid, int64_t rows_pad, float p, uint64_t seed, float *O, int64_t ldo, float *ctx,
                         int64_t ctx_floats, void *stream);
int u2gnn_attn_small_bwd(const float *ctx, int64_t ctx_floats, const float *W_in, int64_t dp, int64_t d,
                         int64_t n_valid, int64_t rows_pad, float p, uint64_t seed, const float *dO, int64_t ld_do,
                         const float *delta, float q_scale, float *dQKV, int64_t ld_dqkv, float *dX, int64_t lddx,
                         float *ws, int64_t ws_floats, void *stream);

/* ---- ABI v15: the row-local tail of a small-width encoder layer (d <= 32, dp = 64), one launch each way ----
 * forward  (a3.3 + a3.4): Z1 = drop1(O W_o^T + b_o) + X, X1 = LayerNorm1(Z1) (mean1, rstd1), Hd = dropff(relu(X1
 *          W1^T + b1)), Z2 = drop2(Hd W2^T + b2) + X1, X2 = LayerNorm2(Z2) (mean2, rstd2) -- exact fp32, one wave
 *          per row; rows >= n_valid and padding columns written 0.
 * backward given dX2 and the forward's tensors: dF = drop2'(LN2^T dX2), dH = (Hd > 0) dF W2 / (1-p), dX1 = LN2^T dX2
 *          + dH W1, dX = LN1^T dX1 (the residual branch; the in-projection's dX product accumulates onto it), dA =
 *          drop1'(dX), dO = dA W_o, delta = rowsum(dO * O).  The parameter gradients are the caller's (column sums
 *          of dF, dH, dA and the LayerNorm terms).
 * Weights in the executor's padded layouts (W_o [dp][dp], W1 [ffp][dp], W2 [dp][ffp], biases zero-padded to dp /
 * ffp; LayerNorm gamma / beta unpadded [d]); activations [rows_pad][dp] (Hd, dH: [rows_pad][ffp]);
 * rows_pad % 8 == 0, ffp % 64 == 0; W_o, W1, O 16-byte aligned. */
typedef struct u2gnn_small_tail_args {
    int64_t n_valid, rows_pad, d, dp, ff, ffp;
    float p, eps;
    uint64_t seed_drop1, seed_dropff, seed_drop2;
    const float *W_o, *b_o, *n1_w, *n1_b, *W1, *b1, *W2, *b2, *n2_w, *n2_b;
    const float *O, *X;                                       /* forward inputs (O also read by the backward) */
    float *Z1, *X1, *mean1, *rstd1, *Hd, *Z2, *X2, *mean2, *rstd2;   /* forward outputs; the backward reads them */
    const float *dX2;                                         /* backward input */
    float *dX1, *dF, *dH, *dX, *dA, *dO, *delta;               /* backward outputs */
} u2gnn_small_tail_args;
int u2gnn_layer_tail_small_fwd(const u2gnn_small_tail_args *a, void *stream);
int u2gnn_layer_tail_small_bwd(const u2gnn_small_tail_args *a, void *stream);

/* ---- ABI v15: a whole small-width encoder layer (d <= 32, dp = 64) -- what the layer executor runs ----------
 * fwd: the in-projection of t->X and the node attention (u2gnn_attn_small_fwd: O into t->O, the attention context
 *      into ctx) and the tail (u2gnn_layer_tail_small_fwd) -- rows_pad >= 1024: attention and tail in ONE launch
 *      (the O row goes from registers into its out-projection), below that as two; 2 or 3 launches.
 * bwd: the tail backward (u2gnn_layer_tail_small_bwd: dX1, dF, dH, dA, dO, delta and the residual dX), then the
 *      attention backward (u2gnn_attn_small_bwd: dQKV and, when accumulate_dx, dX += dQKV W_in) -- rows_pad >= 1024:
 *      the tail backward and the dQ walk in ONE launch, its dO row and delta handed over in LDS; 2 or 3 launches.
 * Same results as the separate calls up to the order of the hidden-unit partial sums of the fused forms. */
int u2gnn_layer_small_fwd(const u2gnn_small_tail_args *t, const float *W_in, const float *b_in, uint64_t attn_seed,
                          float *ctx, int64_t ctx_floats, void *stream);
int u2gnn_layer_small_bwd(const u2gnn_small_tail_args *t, const float *W_in, uint64_t attn_seed, const float *ctx,
                          int64_t ctx_floats, float *dQKV, int64_t ld_dqkv, int32_t accumulate_dx, float *ws,
                          int64_t ws_floats, void *stream);

/* ---- ABI v16: the forward tail (a3.3 + a3.4) of a mid-width layer (d <= 256, dp = rup(d, 64); the layer
 * executor uses it from d > 32 up to rows_pad <= 512: C2's IMDBBINARY batches) -- what five GEMM / LayerNorm
 * launches did (out-projection, LayerNorm1, FFN1, FFN2, LayerNorm2) in two: a row-block x hidden-chunk kernel
 * (out-projection + dropout1 + residual + LayerNorm1, FFN1 + ReLU + dropout for its 128 hidden units, their
 * FFN2 partial sums into chunk slabs in ws) and u2gnn_slab_bias_drop_resid_ln over the ceil(ffp / 128) slabs.
 * Exact fp32 on the vector ALUs, deterministic; rows >= n_valid written as 0 (Z1, X1, Hd, Z2, X2, statistics).
 * Fields as u2gnn_small_tail_args (forward inputs and outputs); rows_pad % 4 == 0; W_o, W1, W2, O, ws 16-byte
 * aligned.  ws: u2gnn_layer_tail_mid_ws_floats floats (-1 for unsupported sizes). */
int64_t u2gnn_layer_tail_mid_ws_floats(int64_t rows_pad, int64_t dp, int64_t ffp);
int u2gnn_layer_tail_mid_fwd(const u2gnn_small_tail_args *t, float *ws, int64_t ws_floats, void *stream);

/* ---- a12: dropout on the concatenated UnSup node embeddings (model_U2GNN_Unsup_multi.py:56) --
 * Y[i, j] = X[i, j] * keep(seed, i, j) / (1-p) for i < rows, j < cols.  The backward is the same
 * call on the upstream gradient with the same seed.  Y may alias X. */
int u2gnn_dropout(const float *X, int64_t ldx, float *Y, int64_t ldy, int64_t rows, int64_t cols, float p,
                  uint64_t seed, void *stream);

/* ---- debugging / tests ---------------------------------------------------------------- */
/* out[i*cols + j] = keep(seed, i, j) ? 1 : 0   (the exact dropout mask the kernels apply) */
int u2gnn_dropout_mask(uint64_t seed, int64_t rows, int64_t cols, float p, uint8_t *out, void *stream);

/* ---- paper-semantics neighbourhood attention ---------------------
 * Token rows node-major (row n*W + s = slot s of node n, W = k+1 <= 32); QKV [rows_pad, ldq >= 3dp]
 * = [Q/sqrt(d) | K | V].  Per node: P = softmax(Qs K^T) over the node's W keys, Pd = dropout(P)
 * (keep(seed, n*W+i, j)), O = Pd V.  Psave [n_nodes, W, W] holds P for the backward.  Rows
 * n_nodes*W .. rows_pad-1 of O (resp. dQKV) are zeroed.  LDS bound: (3W*dp + W(W+1))*4 B (fwd),
 * (4W*dp + 2W(W+1))*4 B (bwd) <= 160 KiB, else U2GNN_E_SHAPE. */
int u2gnn_window_attn_fwd(const float *QKV, int64_t ldq, int32_t W, int32_t dp, float *O, int64_t ldo,
                          float *Psave, float p, uint64_t seed, int64_t n_nodes, int64_t rows_pad,
                          void *stream);
/* dQKV = [q_scale * dL/dQs | dL/dK | dL/dV] from dO [rows_pad, ldo] and Psave. */
int u2gnn_window_attn_bwd(const float *QKV, int64_t ldq, int32_t W, int32_t dp, const float *dO,
                          int64_t ldo, const float *Psave, float p, uint64_t seed, float q_scale,
                          float *dQKV, int64_t ldg, int64_t n_nodes, int64_t rows_pad, void *stream);

/* ---- a3: one encoder layer (TransformerEncoderLayer(d, nhead=1, ff, dropout), post-LN, slot-0
 * rows) issued natively: forward and backward of pytorch_U2GNN_Sup.py:19-21,35 /
 * pytorch_U2GNN_UnSup.py:37-40,57, launch-for-launch the sequence of u2gnn_hip/engine.py.
 * Padded layouts: Np = roundup(N,256) rows for N >= 1024, else roundup(N,128); dp = roundup(d,64),
 * ffp = roundup(ff,64) columns.
 * All buffers are caller-allocated; u2gnn_layer_sizes gives the three sizes (ctx = tensors
 * saved for the backward, fwd/bwd workspaces).  The backward's parameter-gradient work goes to
 * side_stream (NULL: same stream) after the main-stream results it reads; the caller joins the
 * streams before reading grads and must keep X, ctx, dX2 and ws alive until side_stream drains. */
#define U2GNN_LAYER_DEEP_WGRAD 1   /* weight gradients on the 16-deep-K 128x128 tile */
/* precision "mixed" (ABI v5): with precision == U2GNN_PREC_BF16X3, the three attention-backward
 * node-depth products dS = P o (dO V^T - delta), dQ = dS K, dK = dS^T Q run on plain bf16
 * operands (fp32 accumulation); every other product stays bf16x3 */
#define U2GNN_LAYER_ATTN_BWD_BF16 2
/* precision "fwd32" (ABI v14): with precision == U2GNN_PREC_BF16X3, every FORWARD product (in-projection,
 * Q K^T, P V, out-projection, FFN1, FFN2) runs exact fp32 (the three-pass attention forward); the
 * backward stays bf16x3.  The forward's ReLU decisions then carry fp32 rounding only */
#define U2GNN_LAYER_FWD_F32 4
/* precision "fwd6" (ABI v17): with precision == U2GNN_PREC_BF16X3, every FORWARD product runs on the three-plane
 * split U2GNN_PREC_BF16X6 (fp32-accurate products on bf16 MFMA); the backward stays bf16x3.  Excludes FWD_F32 */
#define U2GNN_LAYER_FWD_X6 8
/* precision "fwdh" (ABI v18): with precision == U2GNN_PREC_BF16X3, every FORWARD product runs on the two-plane
 * fp16 split U2GNN_PREC_F16X3 (~2^-21 per product at the bf16x3 rate); the backward stays bf16x3.  Excludes
 * FWD_F32 and FWD_X6 */
#define U2GNN_LAYER_FWD_H3 16
/* ABI v18: with precision U2GNN_PREC_F16X3, a GEMM's x2 output (Cx2) holds fp16 hi / lo of 2^U2GNN_H3_X2_EXP * C in
 * the x2 layout (the in-projection's V block for the f16x3 softmax.P.V, which takes that scale back out) */
#define U2GNN_H3_X2_EXP 6
typedef struct u2gnn_layer_dims {
    int64_t N, d, ff;      /* real rows (nodes; window mode: nodes * window tokens), model width, FFN width */
    int32_t precision;     /* U2GNN_PREC_* */
    int32_t flags;         /* U2GNN_LAYER_* */
    int32_t window;        /* 0: attention over all N rows (the fork's semantics); W >= 1: attention
                              within consecutive windows of W rows (paper semantics, N % W == 0) */
    int32_t reserved;
} u2gnn_layer_dims;
typedef struct u2gnn_layer_params {
    const float *W_in, *b_in, *W_o, *b_o, *W1, *b1, *W2, *b2;   /* padded copies ([3dp,dp], [3dp], ...) */
    const float *n1_w, *n1_b, *n2_w, *n2_b;                      /* LayerNorm affine, real [d] */
} u2gnn_layer_params;
typedef struct u2gnn_layer_seeds {
    float p_drop;          /* 0 in eval mode */
    uint64_t attn, drop1, dropff, drop2;   /* per-site dropout seeds */
} u2gnn_layer_seeds;
typedef struct u2gnn_layer_grads {  /* real-shaped parameter gradients, overwritten */
    float *in_w, *in_b, *out_w, *out_b, *l1_w, *l1_b, *l2_w, *l2_b, *n1_w, *n1_b, *n2_w, *n2_b;
} u2gnn_layer_grads;
int u2gnn_layer_sizes(const u2gnn_layer_dims *dims, float p_drop, int64_t *ctx_bytes,
                      int64_t *fwd_ws_bytes, int64_t *bwd_ws_bytes);
/* X, X2: [Np, dp]; ctx may be NULL when no backward follows (the saved tensors then live in ws,
 * which must be ctx_bytes + fwd_ws_bytes large). */
int u2gnn_layer_fwd(const u2gnn_layer_dims *dims, const u2gnn_layer_params *w,
                    const u2gnn_layer_seeds *s, const float *X, float *X2, void *ctx,
                    int64_t ctx_bytes, void *ws, int64_t ws_bytes, void *stream);
/* dX2, dX: [Np, dp]; X is the forward's input.  dX = NULL: the input gradient is not wanted
 * (first layer of a stack whose input is not trainable) and its in-projection GEMM is skipped. */
int u2gnn_layer_bwd(const u2gnn_layer_dims *dims, const u2gnn_layer_params *w,
                    const u2gnn_layer_seeds *s, const float *X, const void *ctx, int64_t ctx_bytes,
                    const float *dX2, float *dX, const u2gnn_layer_grads *g, void *ws,
                    int64_t ws_bytes, void *stream, void *side_stream);

/* ---- ABI v5: live launch timing of one product of the layer executor (diagnostics) ----
 * u2gnn_probe_arm(role, capacity) creates `capacity` pairs of timing events; every following
 * u2gnn_layer_fwd/bwd launch of that role is bracketed by a pair recorded on the stream the kernel
 * runs on (the first `capacity` launches).  u2gnn_probe_collect waits for the recorded events and
 * returns the summed device time and the launch count, then frees the events.  One probe per
 * process; arm/collect from the thread that issues the layers (bench.py's timed region). */
#define U2GNN_ROLE_QK 1   /* S = Q K^T                                   */
#define U2GNN_ROLE_PV 2   /* O = Pd V (split-K GEMM only, not its reduce; fused path: the softmax.P.V
                             kernel and its combine pass) */
#define U2GNN_ROLE_DS 3   /* dS = P o (dO V^T - delta)                   */
#define U2GNN_ROLE_DV 4
#define U2GNN_ROLE_DQ 5
#define U2GNN_ROLE_DK 6
int u2gnn_probe_arm(int32_t role, int32_t capacity);
int u2gnn_probe_collect(float *total_ms, int32_t *launches);

/* ---- ABI v6: device-resident step state (HIP-graph replay of a training step) ----
 * A captured step replays every launch with its capture-time arguments; the two things that must
 * change from step to step live in device memory instead:
 *  - dropout masks: after u2gnn_set_seed_epoch(epoch) every dropout-drawing kernel launched (gemm
 *    dropout epilogues, softmax, LayerNorm backward, pooling, dropout, window attention) mixes the
 *    device uint64 *epoch into its by-value seed: seed ^ *epoch * 0x9E3779B97F4A7C15 (epoch 0 =
 *    the plain seed).  Per device (ABI v17): the call sets the calling thread's current device's epoch, read at
 *    launch time by launches on that device; NULL switches it off; U2GNN_E_ARG without a current device.
 *  - Adam's bias corrections: u2gnn_adam_dev is u2gnn_adam with step_size = lr / (1 - beta1^t) and
 *    bc2_sqrt = sqrt(1 - beta2^t) formed on the device from the double *lr and the int64 step *t.
 *  u2gnn_step_advance(epoch, t) adds 1 to each non-NULL counter (one single-thread kernel): the first
 *  launch of a captured step. */
int u2gnn_set_seed_epoch(const uint64_t *epoch);
int u2gnn_step_advance(uint64_t *epoch, int64_t *step, void *stream);
int u2gnn_adam_dev(float *param, const float *grad, float *exp_avg, float *exp_avg_sq, int64_t n,
                   const float *sqnorm, float max_norm, double beta1, double beta2, float eps,
                   const double *lr, const int64_t *step, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* U2GNN_HIP_H */
