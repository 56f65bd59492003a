// Node-axis attention for small feature widths (d <= 32: the U2GNN-UnSup encoders, REDDIT-M5K d = 4 (C5),
// PTC d = 19 (C3), MUTAG d = 7 (C1)) -- a3.2 of SURVEY.md §8 and its backward
// (torch MHA inside pytorch_U2GNN_UnSup.py:37-40,57 / pytorch_U2GNN_Sup.py:19-21,35).
//
// At d <= 32 the matrix-core path pads every attention product to dp = 64 columns (94 % padding at d = 4)
// and still moves the N x N score and probability images through HBM several times per layer.  Here the
// N^2 work runs in exact fp32 on the vector ALUs and nothing N x N is ever stored (flash-style), in four
// launches per layer, each writing its final outputs (no partial buffers, no combine launches):
//   proj     the in-projection (a3.1) of the layer input straight into the compact context (layouts below):
//            no [Np][3 dp] image, no matrix-core launch for a d x 3d product;
//   forward  SA_SPL = 2 waves per query row, the 64 lanes of each splitting its half of every LDS key tile
//            (two consecutive keys per lane per 128-key round): scores, an online max / sum-exp rescale per
//            8 keys, the dropout hash (one finaliser per key pair) and o += e v; the lanes merge by a
//            butterfly, the two waves through LDS; lane c writes column c of O = sum_kept e v / (L (1 - p))
//            and lane 0 the row statistics (M, 1/L) the backward recomputes P = exp2(s log2e - M) / L from;
//   dQ       the same row walk: dS_ij = P_ij (keep dO_i.V_j / (1 - p) - delta_i), dQ_i += dS_ij K_j; each
//            row also writes its compact record (Q, dO, M, 1/L, delta, row key) for
//   dK, dV   SA_SPL waves per key row, the lanes splitting LDS tiles of query records:
//            dV_j += Pd_ij dO_i, dK_j += dS_ij Q_i; then the in-projection's dX_j += dQKV_j W_in (row-local).
// Softmax semantics are the reference's: softmax over the keys, THEN dropout(p) on the probabilities with
// 1/(1-p) scaling, THEN the product with V (torch SDPA math path); delta_i = rowsum(dO_i * O_i) as for the
// matrix-core path.  The keep decisions are u2gnn_keep(seed, i, j, p), the hash every dropout site uses.
// Deterministic: fixed key / query partition and butterfly merges in a fixed order.
#include <cmath>
#include <cstring>

#include "u2gnn_common.h"

// Phase stamps of the fused kernels (experiment builds only: -DSX_STAMPS, tools/sl_stamps.py): thread 0 of a
// workgroup records the constant-rate wall clock (100 MHz) at phase boundaries; read back by u2gnn_dbg_sx_stamps.
#ifdef SX_STAMPS
__device__ unsigned long long g_sx_stamps[2][4096][16];
#define SX_STAMP(kern, k)                                                                                            \
    do {                                                                                                           \
        if (threadIdx.x == 0 && blockIdx.x < 4096) g_sx_stamps[kern][blockIdx.x][k] = (unsigned long long)wall_clock64(); \
    } while (0)
#else
#define SX_STAMP(kern, k) \
    do {                  \
    } while (0)
#endif

#ifndef SX_BWD_ORDER
#define SX_BWD_ORDER 1
#endif

namespace {

constexpr int SA_WAVES = 8;    // rows (forward, dQ) or key rows (dK / dV) per 512-thread workgroup
constexpr int SA_NT = 64 * SA_WAVES;
// keys (forward, dQ) / queries (dK, dV) staged in LDS per tile: 32 KB of K and V (16-34 KB of query
// records): two to four workgroups per CU
#ifndef SA_KT4_F
#define SA_KT4_F 0   // (A/B: key-tile size of the DM = 4 forward / dQ walks; 0 = the formula below)
#endif
#ifndef SA_KT4_B
#define SA_KT4_B 0   // (A/B: query-tile size of the DM = 4 dK / dV walk)
#endif
template <int DM> constexpr int sa_kt_f() {   // 128-key rounds per wave
    return DM == 4 && SA_KT4_F ? SA_KT4_F : 4096 / DM > 256 ? 4096 / DM / 256 * 256 : 256;
}
template <int DM> constexpr int sa_kt_b() {   // 64-query rounds per wave
    return DM == 4 && SA_KT4_B ? SA_KT4_B : 2048 / DM > 128 ? 2048 / DM / 128 * 128 : 128;
}
constexpr float SA_LOG2E = 1.4426950408889634f;
// 2^x as one v_exp_f32: exp2f adds a 6-instruction rescue of results below 2^-126 (round 6: the walks are
// VALU-issue-bound, SQ_INSTS_VALU); softmax terms that small are flushed to 0 -- they are below fp32 resolution of
// the row sums they would join (every row sum holds its maximum term, exp2(0) = 1).  exp2(-inf) = 0 as before.
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }
// waves per SIMD the register budget is sized for: 4 (128 VGPRs) up to DM = 16, 2 (256) beyond, where the row's
// q, o / dq / dk, dv arrays alone take 2-3 DM registers (the 128 cap spilled them to scratch)
template <int DM> constexpr int sa_min_waves() { return DM <= 8 ? 4 : 2; }

// Layouts (all fp32; DM = d rounded up to a multiple of 4 up to 24, else 32):
//   ctx (the forward's saved context, u2gnn_attn_small_ctx_floats):  st [Np][2] = (M in log2 units, 1/L) |
//        qc [Np][DM] (Q, pre-scaled) | kvc [Np][2 DM] (K then V of a row, adjacent); rows >= N all zero.
//        Every workgroup stages the keys from 2 DM contiguous floats per key (round 5, first form: a strided
//        [Np][3 dp] image cost two 16-byte pieces of two far-apart cache lines per key and workgroup).
//   ws (the backward's scratch, u2gnn_attn_small_ws_floats): rq [Np][RQ], RQ = 2 DM + 4:
//        Q[DM], dO[DM], M, 1/L, delta, row key -- written by the dQ launch for its own rows, staged by dK / dV.
struct SaP {
    const float *x;     // forward: the layer input [Np][ldx] (d real columns)
    int64_t ldx;
    const float *w_in;  // the in-projection [3 dp][dp] (padded; rows c, dp + c, 2 dp + c: Q, K, V column c)
    const float *b_in;  // [3 dp]
    int32_t dp, d, N, Np;
    float p;
    uint64_t seed;
    const uint64_t *epoch;
    float *ctx;         // st | qc | kvc
    const float *dO;    // backward: [Np][ld_do]
    int64_t ld_do;
    const float *delta; // backward: [Np]
    float *rq;          // backward: [Np][RQ]
    float *out;         // forward: O; backward: dQKV
    int64_t ld_out;
    float q_scale;      // 1/sqrt(d): Q's scale in the forward, dQ's in the backward
    float *dx;          // backward: dX += dQKV W_in (nullptr: not wanted)
    int64_t lddx;
};

template <int DM> __host__ __device__ constexpr int sa_rq() { return 2 * DM + 4; }

// 16 bytes from p (a valid, clamped address), zeroed where !ok -- the load is issued whatever ok is
__device__ __forceinline__ float4 ld4z(const float *p, bool ok) {
    const float4 t = *reinterpret_cast<const float4 *>(p);
    return make_float4(ok ? t.x : 0.f, ok ? t.y : 0.f, ok ? t.z : 0.f, ok ? t.w : 0.f);
}
__host__ __device__ inline float *sa_st(float *ctx) { return ctx; }
template <int DM> __host__ __device__ inline float *sa_qc(float *ctx, int64_t Np) { return ctx + 2 * Np; }
template <int DM> __host__ __device__ inline float *sa_kvc(float *ctx, int64_t Np) { return ctx + (2 + DM) * Np; }

template <int DM>
__device__ __forceinline__ void load_row(const float *src, float (&x)[DM]) {
#pragma unroll
    for (int c = 0; c < DM; c += 4) {
        const float4 v = *reinterpret_cast<const float4 *>(src + c);
        x[c] = v.x, x[c + 1] = v.y, x[c + 2] = v.z, x[c + 3] = v.w;
    }
}

template <int DM>
__device__ __forceinline__ void store_row(float *dst, const float (&x)[DM]) {
#pragma unroll
    for (int c = 0; c < DM; c += 4) *reinterpret_cast<float4 *>(dst + c) = make_float4(x[c], x[c + 1], x[c + 2], x[c + 3]);
}

template <int DM>
__device__ __forceinline__ float dot_lds(const float (&x)[DM], const float *y) {
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < DM; c += 4) {
        const float4 v = *reinterpret_cast<const float4 *>(y + c);
        s = fmaf(x[c], v.x, s);
        s = fmaf(x[c + 1], v.y, s);
        s = fmaf(x[c + 2], v.z, s);
        s = fmaf(x[c + 3], v.w, s);
    }
    return s;
}

// lane c of a wave writes column c (< width) of a row: x[c] for c < d, 0 beyond (x is the same in every lane)
template <int DM>
__device__ __forceinline__ float lane_col(const float (&x)[DM], int c) {
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < DM; ++k) v = c == k ? x[k] : v;
    return v;
}

// Work split inside a 512-thread workgroup: SA_RB rows (forward, dQ: query rows; dK / dV: key rows), each
// taken by SA_SPL waves that split the tile between them (wave s: the s-th part), lanes splitting each part;
// a row's partial results merge across its lanes (butterfly) and then across its waves (LDS).
#ifndef SA_SPL_
#define SA_SPL_ 2   // (A/B: -DSA_SPL_=1 builds one wave per row, 8 rows per workgroup)
#endif
constexpr int SA_SPL = SA_SPL_, SA_RB = SA_WAVES / SA_SPL;
// the fused forward (attention + tail, rows_pad >= 1024) at DM = 4 takes one wave per row, 8 rows per workgroup: half the
// workgroups, each staging the keys and the weight chunk once for 8 rows (round 6, C5 shape: 16.7 vs 18.0 us at
// N = 1 914, 30.2 vs 38.5 at 3 900 per layer forward; the backward keeps 2, tools/small_layer_bench.py)
#ifndef SA_FWD_SPL_
#define SA_FWD_SPL_ 1
#endif
constexpr int SA_FWD_SPL = SA_FWD_SPL_;
#ifndef SA_BWD_SPL_
#define SA_BWD_SPL_ 2   // (A/B: 1 = the fused tail backward + dQ walk at one wave per row, SA_BWD_MINW waves per SIMD)
#endif
#ifndef SA_BWD_MINW
#define SA_BWD_MINW 2
#endif
constexpr int SA_BWD_SPL = SA_BWD_SPL_;

// Staging of records [t0, t0 + KT) of a compact [Np][W] array (W = WA + WB + WC, each a multiple of 4) into the
// LDS arrays a [KT][WA], b [KT][WB], c [KT][WC]; records at or past Np are zeros.  PS (pair split): record t goes to
// row ps_row(t) = (t & 1) KT / 2 + t / 2, so a lane walking the key pair (2 c, 2 c + 1) with c = base + lane reads
// two rows that are consecutive across the lanes (16-byte stride at DM = 4: no LDS bank conflicts; the natural
// order put the lanes 32 bytes apart).  In two halves: tile_load
// issues every global load of the tile into registers (SA_PER float4 per thread, all in flight together) and
// tile_store writes them to LDS -- so the next tile's loads run under this tile's compute, and a tile costs one
// load latency instead of one per loop iteration (a load -> ds_write loop waits on every load).
template <int KT> __device__ __forceinline__ int ps_row(int t) { return (t & 1) * (KT / 2) + (t >> 1); }

template <int KT, int WA, int WB, int WC, bool PS = false>
struct Tile {
    static constexpr int W4 = (WA + WB + WC) / 4, NE = KT * W4, PER = (NE + SA_NT - 1) / SA_NT;
    float4 v[PER];
    __device__ __forceinline__ void load(const float *src, int t0, int Np) {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int e = threadIdx.x + i * SA_NT, t = e / W4;
            v[i] = make_float4(0.f, 0.f, 0.f, 0.f);   // (a branch, not "cond ? *p : z": no private copy of z)
            if (e < NE && t0 + t < Np) v[i] = *reinterpret_cast<const float4 *>(src + (int64_t)t0 * (4 * W4) + 4 * (int64_t)e);
        }
    }
    __device__ __forceinline__ void store(float (*a)[WA], float (*b)[WB], float *c) const {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int e = threadIdx.x + i * SA_NT;
            if (e >= NE) break;
            const int t = PS ? ps_row<KT>(e / W4) : e / W4, k = 4 * (e % W4);
            if (k < WA) *reinterpret_cast<float4 *>(&a[t][k]) = v[i];
            else if (k < WA + WB) *reinterpret_cast<float4 *>(&b[t][k - WA]) = v[i];
            else *reinterpret_cast<float4 *>(c + t * WC + k - WA - WB) = v[i];
        }
    }
};

// ---- a3.1 in-projection straight into the compact context: (Q, K, V) = X W_in^T + b_in, Q scaled by 1/sqrt(d)
// (the bias epilogue's order: (acc + b) * scale); rows >= N zero.  One thread per 4 output columns of a row.
template <int DM>
__global__ void __launch_bounds__(256) sa_proj_kernel(SaP P) {
    constexpr int C4 = DM / 4;
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= (int64_t)P.Np * 3 * C4) return;
    const int r = (int)(e / (3 * C4)), bc = (int)(e % (3 * C4)), b = bc / C4, c = 4 * (bc % C4);
    float o[4] = {0.f, 0.f, 0.f, 0.f};
    if (r < P.N) {
        float xv[DM];
        load_row<DM>(P.x + (int64_t)r * P.ldx, xv);   // columns d .. DM of the padded row are zero
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int64_t wr = (int64_t)b * P.dp + c + q;   // W_in row of output column c + q of block b
            float w[DM];
            load_row<DM>(P.w_in + wr * P.dp, w);
            float acc = 0.f;
#pragma unroll
            for (int k = 0; k < DM; ++k) acc = fmaf(xv[k], w[k], acc);
            o[q] = acc + P.b_in[wr];
            if (b == 0) o[q] *= P.q_scale;
        }
    }
    float *dst = b == 0 ? sa_qc<DM>(P.ctx, P.Np) + (int64_t)r * DM + c
                        : sa_kvc<DM>(P.ctx, P.Np) + (int64_t)r * 2 * DM + (b - 1) * DM + c;
    *reinterpret_cast<float4 *>(dst) = make_float4(o[0], o[1], o[2], o[3]);
}

// the row-local tail's launch shape and parameters (its kernels: second half of this file)
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

template <int DM, int HC, bool BIAS> struct Stage;
template <int DM> struct TailRowF;
template <int DM> struct TailRowB;
template <int DM, int SPL = SA_SPL> constexpr int ls_nw() { return (ls_hc<DM>() / 64 + SPL - 1) / SPL; }   // units per lane per chunk
template <int DM, int SPL>
__device__ void tail_hd_load(const LsP &T, int i, int sp, int h0, float (&hvs)[ls_nw<DM, SPL>()]);
template <int DM, int SPL> __device__ void tail_fwd_rows(const LsP &T, int i, int rw, int sp, const float (&of)[DM],
                                                         bool fin, const TailRowF<DM> &rp,
                                                         Stage<DM, ls_hc<DM>(), true> &sg, float *smem);
template <int DM, int SPL> __device__ void tail_bwd_rows(const LsP &T, int i, int rw, int sp, bool fin,
                                                         const TailRowB<DM> &rp, Stage<DM, ls_hc<DM>(), false> &sg,
                                                         float (&hvs)[ls_nw<DM, SPL>()], float (&g)[DM], float &dl,
                                                         float *smem);
template <int DM, int SPL = SA_SPL> constexpr int tail_smem_floats();

// ---- forward: one query row per SA_SPL waves -------------------------------------------------------------
// TAIL (ABI u2gnn_layer_small_fwd, rows_pad >= 1024): the same workgroup then runs the row-local tail of its
// SA_RB rows (tail_fwd_rows): the attention output O never makes a round trip before its out-projection
template <int DM, bool TAIL, int SPL = SA_SPL>
__global__ void __launch_bounds__(SA_NT, sa_min_waves<DM>()) sa_fwd_kernel(SaP P, LsP T) {
    constexpr int RB = SA_WAVES / SPL;   // rows per workgroup
    constexpr int SA_KT = sa_kt_f<DM>();
    constexpr int PART = SA_KT / SPL, NP = PART / 128;   // keys per wave per tile; key pairs per lane
    // keys per lane between rescales (their K rows are live in registers), at most the wave's part of the tile
    // (2 NP keys per lane): a larger chunk would index ks past the tile for DM >= 8
    constexpr int CU = (DM <= 8 ? 8 : 4) < 2 * NP ? (DM <= 8 ? 8 : 4) : 2 * NP;
    static_assert(NP >= 1 && PART % 128 == 0, "a wave's part of the key tile: whole 128-key rounds");
    __shared__ __attribute__((aligned(16))) float ks[SA_KT][DM];
    __shared__ __attribute__((aligned(16))) float vs[SA_KT][DM];
    __shared__ float xw[RB][SPL][2 + DM];
    const uint64_t seed = u2gnn_seed(P.seed, P.epoch);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, rw = w % RB, sp = w / RB;
    const int i = blockIdx.x * RB + rw;
    const bool live = i < P.N;
    const float *kvc = sa_kvc<DM>(P.ctx, P.Np);
    float q[DM], o[DM];
#pragma unroll
    for (int c = 0; c < DM; ++c) q[c] = o[c] = 0.f;
    if (live) load_row<DM>(sa_qc<DM>(P.ctx, P.Np) + (int64_t)i * DM, q);
    const bool drop = P.p > 0.f;
    const uint32_t thr = u2gnn_keep_thr(P.p), rk = u2gnn_row_key(seed, (uint32_t)i);
    float m = -INFINITY, l = 0.f;
    if (TAIL) SX_STAMP(0, 0);
    Tile<SA_KT, DM, DM, 0, true> tl;
    tl.load(kvc, 0, P.Np);
    [[maybe_unused]] TailRowF<DM> rp;   // TAIL: the row operands of the tail, in flight under the walk
    if constexpr (TAIL)
        if (sp == 0) rp.load(T, i);
    for (int t0 = 0; t0 < P.N; t0 += SA_KT) {
        __syncthreads();
        tl.store(ks, vs, nullptr);
        __syncthreads();
        if (TAIL && t0 == 0) SX_STAMP(0, 1);
        if (t0 + SA_KT < P.N) tl.load(kvc, t0 + SA_KT, P.Np);   // the next tile, in flight under this one
        if (!live) continue;
        // this wave's keys of the tile: pairs (t0 + sp PART + 128 h + 2 lane, +1), LDS rows ps_row; CU / 2 pairs per
        // rescale
#pragma unroll 1
        for (int h0 = 0; h0 < NP; h0 += CU / 2) {
            float s[CU];
            float cm = -INFINITY;
#pragma unroll
            for (int u = 0; u < CU; ++u) {
                const int t = sp * PART + 128 * (h0 + u / 2) + 2 * lane + (u & 1);
                const float x = dot_lds<DM>(q, ks[ps_row<SA_KT>(t)]) * SA_LOG2E;   // rows past N are zeros: finite
                s[u] = (h0 + u / 2 < NP && t0 + t < P.N) ? x : -INFINITY;
                cm = fmaxf(cm, s[u]);
            }
            if (cm == -INFINITY) continue;   // none of this lane's keys in the chunk
            const float mn = fmaxf(m, cm);
            const float sc = fexp2(m - mn);  // m = -inf: 0
            l *= sc;
#pragma unroll
            for (int c = 0; c < DM; ++c) o[c] *= sc;
#pragma unroll
            for (int u = 0; u < CU; u += 2) {
                const int t = sp * PART + 128 * (h0 + u / 2) + 2 * lane;
                bool k0 = true, k1 = true;
                if (drop) {
                    const uint32_t hh = u2gnn_pair_hash(rk, (uint32_t)(t0 + t) >> 1);
                    k0 = u2gnn_keep_lo(hh, thr), k1 = u2gnn_keep_hi(hh, thr);
                }
                const float e0 = fexp2(s[u] - mn), e1 = fexp2(s[u + 1] - mn);   // 0 past N
                l += e0 + e1;
                const float a0 = k0 ? e0 : 0.f, a1 = k1 ? e1 : 0.f;
                const int tt = ps_row<SA_KT>(h0 + u / 2 < NP ? t : 0);   // (a0 = a1 = 0 there)
#pragma unroll
                for (int c = 0; c < DM; ++c) o[c] = fmaf(a1, vs[tt + SA_KT / 2][c], fmaf(a0, vs[tt][c], o[c]));
            }
            m = mn;
        }
    }
    if (TAIL) SX_STAMP(0, 2);
    // TAIL: the tail's first weight chunk, in flight under the merge and the out-projection / LayerNorm1
    [[maybe_unused]] Stage<DM, ls_hc<DM>(), true> sg;
    if constexpr (TAIL) sg.load(T, 0);
    // merge of the 64 lanes' (m, l, o): the wave's maximum first, each lane rescales to it once, then plain
    // butterfly sums (one exp per lane instead of two per butterfly level); every lane ends with the same values
    {
        const float M = wave_max(m);
        const float f = m == -INFINITY ? 0.f : fexp2(m - M);   // (M = -inf only with every lane empty)
        l = wave_sum(l * f);
#pragma unroll
        for (int c = 0; c < DM; ++c) o[c] = wave_sum(o[c] * f);
        m = M;
    }
    // then the row's SPL waves, in wave order
    if (lane == 0) {
        xw[rw][sp][0] = m;
        xw[rw][sp][1] = l;
#pragma unroll
        for (int c = 0; c < DM; ++c) xw[rw][sp][2 + c] = o[c];
    }
    __syncthreads();
    if (TAIL) SX_STAMP(0, 3);
    const bool fin = sp == 0 && i < P.Np;   // the row's finishing wave
    if (!TAIL && !fin) return;
    float of[DM];   // fin: the row of O
#pragma unroll
    for (int c = 0; c < DM; ++c) of[c] = 0.f;
    if (fin) {
        float M = xw[rw][0][0];
#pragma unroll
        for (int x = 1; x < SPL; ++x) M = fmaxf(M, xw[rw][x][0]);
        float L = 0.f;
#pragma unroll
        for (int c = 0; c < DM; ++c) o[c] = 0.f;
        if (M != -INFINITY) {
#pragma unroll
            for (int x = 0; x < SPL; ++x) {
                const float f = xw[rw][x][0] == -INFINITY ? 0.f : fexp2(xw[rw][x][0] - M);
                L = fmaf(xw[rw][x][1], f, L);
#pragma unroll
                for (int c = 0; c < DM; ++c) o[c] = fmaf(xw[rw][x][2 + c], f, o[c]);
            }
        }
        const float invL = live && L > 0.f ? 1.f / L : 0.f;
        const float s1p = drop ? 1.f / (1.f - P.p) : 1.f;
#pragma unroll
        for (int c = 0; c < DM; ++c) of[c] = (live && c < P.d) ? o[c] * invL * s1p : 0.f;
        float *orow = P.out + (int64_t)i * P.ld_out;
        for (int c = lane; c < P.dp; c += 64) orow[c] = lane_col<DM>(of, c);
        if (lane == 0) {
            float *st = sa_st(P.ctx);
            st[2 * (int64_t)i] = live ? M : 0.f;
            st[2 * (int64_t)i + 1] = invL;
        }
    }
    if constexpr (TAIL) {
        SX_STAMP(0, 4);
        __shared__ __attribute__((aligned(16))) float tsm[tail_smem_floats<DM, SPL>()];
        tail_fwd_rows<DM, SPL>(T, i, rw, sp, of, fin, rp, sg, tsm);
        SX_STAMP(0, 9);
    }
}

// ---- backward dQ: one query row per SA_SPL waves; also the row's record for dK / dV -----------------------
// TAIL (ABI u2gnn_layer_small_bwd, rows_pad >= 1024): the workgroup first runs the row-local tail backward of
// its SA_RB rows (tail_bwd_rows), whose dO row and delta then feed the dQ walk from LDS
template <int DM, bool TAIL, int SPL = SA_SPL>
__global__ void __launch_bounds__(SA_NT, SPL == 1 ? SA_BWD_MINW : sa_min_waves<DM>()) sa_bwd_q_kernel(SaP P,
                                                                                                         LsP T) {
    constexpr int RB = SA_WAVES / SPL;   // rows per workgroup
    constexpr int SA_KT = sa_kt_f<DM>();
    constexpr int PART = SA_KT / SPL, NP = PART / 128;
    static_assert(NP >= 1 && PART % 128 == 0, "a wave's part of the key tile: whole 128-key rounds");
    __shared__ __attribute__((aligned(16))) float ks[SA_KT][DM];
    __shared__ __attribute__((aligned(16))) float vs[SA_KT][DM];
    __shared__ float xw[RB][SPL][DM];
    const uint64_t seed = u2gnn_seed(P.seed, P.epoch);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, rw = w % RB, sp = w / RB;
    const int i = blockIdx.x * RB + rw;
    const bool live = i < P.N;
    const float *st = sa_st(P.ctx);
    float q[DM], g[DM], dq[DM];
    float M = 0.f, iL = 0.f, dl = 0.f;
#pragma unroll
    for (int c = 0; c < DM; ++c) q[c] = g[c] = dq[c] = 0.f;
    if constexpr (TAIL) {   // dO and delta of the row from the tail backward (every wave of the row)
        SX_STAMP(1, 0);
        __shared__ __attribute__((aligned(16))) float tsm[tail_smem_floats<DM, SPL>()];
        const bool fin = sp == 0 && i < P.Np;
        Stage<DM, ls_hc<DM>(), false> sg;   // every operand of the tail's first chunk, issued together
        float hvs[ls_nw<DM, SPL>()];
        TailRowB<DM> rp;
        rp.load(T, i);   // (every wave: the LayerNorm2^T operands are the first loads in flight)
#if SX_BWD_ORDER
        __builtin_amdgcn_sched_barrier(0);
#endif
        sg.load(T, 0);
        tail_hd_load<DM, SPL>(T, i, sp, 0, hvs);
        tail_bwd_rows<DM, SPL>(T, i, rw, sp, fin, rp, sg, hvs, g, dl, tsm);
        SX_STAMP(1, 1);
    }
    if (live) {
        load_row<DM>(sa_qc<DM>(P.ctx, P.Np) + (int64_t)i * DM, q);
        if constexpr (!TAIL) {
            load_row<DM>(P.dO + (int64_t)i * P.ld_do, g);
            dl = P.delta[i];
        }
        M = st[2 * (int64_t)i], iL = st[2 * (int64_t)i + 1];
    }
    const bool drop = P.p > 0.f;
    const float s1p = drop ? 1.f / (1.f - P.p) : 1.f;
    const uint32_t thr = u2gnn_keep_thr(P.p), rk = u2gnn_row_key(seed, (uint32_t)i);
    if (sp == 0 && lane == 0 && i < P.Np) {   // the row's record (iL = 0 past N: the dK / dV sweep skips it)
        float *r = P.rq + (int64_t)i * sa_rq<DM>();
        store_row<DM>(r, q);
        store_row<DM>(r + DM, g);
        *reinterpret_cast<float4 *>(r + 2 * DM) = make_float4(M, iL, dl, __uint_as_float(rk));
    }
    const float *kvc = sa_kvc<DM>(P.ctx, P.Np);
    Tile<SA_KT, DM, DM, 0, true> tl;
    tl.load(kvc, 0, P.Np);
    for (int t0 = 0; t0 < P.N; t0 += SA_KT) {
        __syncthreads();
        tl.store(ks, vs, nullptr);
        __syncthreads();
        if (TAIL && t0 == 0) SX_STAMP(1, 2);
        if (t0 + SA_KT < P.N) tl.load(kvc, t0 + SA_KT, P.Np);
        if (!live) continue;
#pragma unroll 2
        for (int h = 0; h < NP; ++h) {
            const int t = sp * PART + 128 * h + 2 * lane;
            bool kp0 = true, kp1 = true;
            if (drop) {
                const uint32_t hh = u2gnn_pair_hash(rk, (uint32_t)(t0 + t) >> 1);
                kp0 = u2gnn_keep_lo(hh, thr), kp1 = u2gnn_keep_hi(hh, thr);
            }
#pragma unroll
            for (int x = 0; x < 2; ++x) {
                const int r = x * (SA_KT / 2) + (t >> 1);   // ps_row(t + x)
                // rows past N are zeros in LDS: their pr is masked to 0 below
                const float pr = t0 + t + x < P.N ? fexp2(dot_lds<DM>(q, ks[r]) * SA_LOG2E - M) * iL : 0.f;
                const float ds = pr * (((x ? kp1 : kp0) ? dot_lds<DM>(g, vs[r]) * s1p : 0.f) - dl);
#pragma unroll
                for (int c = 0; c < DM; ++c) dq[c] = fmaf(ds, ks[r][c], dq[c]);
            }
        }
    }
    if (TAIL) SX_STAMP(1, 3);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1)
#pragma unroll
        for (int c = 0; c < DM; ++c) dq[c] += __shfl_xor(dq[c], off, 64);
    if (lane == 0)
#pragma unroll
        for (int c = 0; c < DM; ++c) xw[rw][sp][c] = dq[c];
    __syncthreads();
    if (sp != 0 || i >= P.Np) return;
#pragma unroll
    for (int c = 0; c < DM; ++c) {
        float t = xw[rw][0][c];
#pragma unroll
        for (int x = 1; x < SPL; ++x) t += xw[rw][x][c];
        dq[c] = t;
    }
    float *row = P.out + (int64_t)i * P.ld_out;   // the Q block of dQKV
    for (int c = lane; c < P.dp; c += 64) row[c] = (live && c < P.d) ? lane_col<DM>(dq, c) * P.q_scale : 0.f;
    if (TAIL) SX_STAMP(1, 4);
}

// ---- backward dK, dV: SA_SPL waves per KP key rows, the waves and lanes splitting the queries -------------
// KP = 2 for DM <= 8: a wave takes the key pair (2j', 2j'+1), so one dropout hash per (query, pair) gives both
// keep bits and each staged query record is read once for both keys
#ifndef SA_KP_SMALL
#define SA_KP_SMALL 2   // (A/B: -DSA_KP_SMALL=1 builds one key row per wave for every width)
#endif
template <int DM> constexpr int sa_kp() { return DM <= 8 ? SA_KP_SMALL : 1; }

template <int DM>
__global__ void __launch_bounds__(SA_NT, sa_min_waves<DM>()) sa_bwd_kv_kernel(SaP P) {
    constexpr int SA_KT = sa_kt_b<DM>(), KP = sa_kp<DM>();
    constexpr int PART = SA_KT / SA_SPL, NU = PART / 64;   // queries per lane per tile
    static_assert(NU >= 1 && PART % 64 == 0, "a wave's part of the query tile: whole 64-query rounds");
    __shared__ __attribute__((aligned(16))) float qs[SA_KT][DM];
    __shared__ __attribute__((aligned(16))) float gs[SA_KT][DM];   // dO rows
    __shared__ __attribute__((aligned(16))) float rs[SA_KT][4];    // M, 1/L, delta, row key (bits)
    __shared__ float xw[SA_RB][SA_SPL][2 * KP * DM];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, rw = w % SA_RB, sp = w / SA_RB;
    const int j0 = (blockIdx.x * SA_RB + rw) * KP;
    const bool live = j0 < P.N;
    float k[KP][DM], v[KP][DM], dk[KP][DM], dv[KP][DM];
#pragma unroll
    for (int x = 0; x < KP; ++x)
#pragma unroll
        for (int c = 0; c < DM; ++c) k[x][c] = v[x][c] = dk[x][c] = dv[x][c] = 0.f;
#pragma unroll
    for (int x = 0; x < KP; ++x)
        if (j0 + x < P.N) {
            const float *kv = sa_kvc<DM>(P.ctx, P.Np) + (int64_t)(j0 + x) * 2 * DM;
            load_row<DM>(kv, k[x]);
            load_row<DM>(kv + DM, v[x]);
        }
    const bool drop = P.p > 0.f;
    const float s1p = drop ? 1.f / (1.f - P.p) : 1.f;
    const uint32_t thr = u2gnn_keep_thr(P.p), jc = (uint32_t)j0 >> 1;
    const bool odd = j0 & 1;   // (KP = 2: j0 even)
    Tile<SA_KT, DM, DM, 4> tl;
    tl.load(P.rq, 0, P.Np);
    for (int t0 = 0; t0 < P.N; t0 += SA_KT) {
        __syncthreads();
        tl.store(qs, gs, &rs[0][0]);
        __syncthreads();
        if (t0 + SA_KT < P.N) tl.load(P.rq, t0 + SA_KT, P.Np);
        if (!live) continue;
#pragma unroll 2
        for (int u = 0; u < NU; ++u) {
            const int t = sp * PART + 64 * u + lane;
            bool kp[KP];
            if (drop) {
                const uint32_t hh = u2gnn_pair_hash(__float_as_uint(rs[t][3]), jc);
                if (KP == 2) kp[0] = u2gnn_keep_lo(hh, thr), kp[KP - 1] = u2gnn_keep_hi(hh, thr);
                else kp[0] = odd ? u2gnn_keep_hi(hh, thr) : u2gnn_keep_lo(hh, thr);
            } else {
#pragma unroll
                for (int x = 0; x < KP; ++x) kp[x] = true;
            }
            float qt[DM], gt[DM];
            load_row<DM>(qs[t], qt);
            load_row<DM>(gs[t], gt);
            const float4 r = *reinterpret_cast<const float4 *>(rs[t]);   // M, 1/L, delta, key
#pragma unroll
            for (int x = 0; x < KP; ++x) {
                // 1/L = 0 for queries past N (their records, and the zero fill past Np): pr = 0
                float sq = 0.f, sg = 0.f;
#pragma unroll
                for (int c = 0; c < DM; ++c) sq = fmaf(k[x][c], qt[c], sq), sg = fmaf(v[x][c], gt[c], sg);
                const float pr = fexp2(sq * SA_LOG2E - r.x) * r.y;
                const float ds = pr * ((kp[x] ? sg * s1p : 0.f) - r.z);
                const float pd = kp[x] ? pr * s1p : 0.f;
#pragma unroll
                for (int c = 0; c < DM; ++c) {
                    dv[x][c] = fmaf(pd, gt[c], dv[x][c]);
                    dk[x][c] = fmaf(ds, qt[c], dk[x][c]);
                }
            }
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1)
#pragma unroll
        for (int x = 0; x < KP; ++x)
#pragma unroll
            for (int c = 0; c < DM; ++c) {
                dk[x][c] += __shfl_xor(dk[x][c], off, 64);
                dv[x][c] += __shfl_xor(dv[x][c], off, 64);
            }
    if (lane == 0)
#pragma unroll
        for (int x = 0; x < KP; ++x)
#pragma unroll
            for (int c = 0; c < DM; ++c) xw[rw][sp][2 * x * DM + c] = dk[x][c], xw[rw][sp][(2 * x + 1) * DM + c] = dv[x][c];
    __syncthreads();
    if (sp != 0) return;
#pragma unroll
    for (int x = 0; x < KP; ++x) {
        const int j = j0 + x;
        if (j >= P.Np) break;
#pragma unroll
        for (int c = 0; c < DM; ++c) {
            float a = xw[rw][0][2 * x * DM + c], b = xw[rw][0][(2 * x + 1) * DM + c];
#pragma unroll
            for (int y = 1; y < SA_SPL; ++y) a += xw[rw][y][2 * x * DM + c], b += xw[rw][y][(2 * x + 1) * DM + c];
            dk[x][c] = a, dv[x][c] = b;
        }
        float *row = P.out + (int64_t)j * P.ld_out;
        for (int c = lane; c < P.dp; c += 64) {
            const bool col = j < P.N && c < P.d;
            row[P.dp + c] = col ? lane_col<DM>(dk[x], c) : 0.f;
            row[2 * P.dp + c] = col ? lane_col<DM>(dv[x], c) : 0.f;
        }
        // the in-projection's input gradient, row j: dX += dQ W_q + dK W_k + dV W_v (dQ of this row written by
        // the dQ launch before this one); lane c < d, W_in's columns read across the lanes
        if (P.dx && j < P.N && lane < P.d) {
            float dq[DM];
            load_row<DM>(row, dq);
            float acc = 0.f;
            const float *wq = P.w_in + lane, *wk = wq + (int64_t)P.dp * P.dp, *wv = wk + (int64_t)P.dp * P.dp;
#pragma unroll
            for (int k = 0; k < DM; ++k) {
                acc = fmaf(dq[k], wq[(int64_t)k * P.dp], acc);
                acc = fmaf(dk[x][k], wk[(int64_t)k * P.dp], acc);
                acc = fmaf(dv[x][k], wv[(int64_t)k * P.dp], acc);
            }
            P.dx[(int64_t)j * P.lddx + lane] += acc;
        }
    }
}

// the register / LDS width of a row: d rounded up to a multiple of 4 up to 24 (PTC d = 19 -> 20), else 32
int sa_dm(int64_t d) { return d < 1 ? 0 : d <= 24 ? (int)((d + 3) / 4 * 4) : d <= 32 ? 32 : 0; }

bool al16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

int sa_check(int64_t dp, int64_t d, int64_t N, int64_t Np, float p, const float *ctx, int64_t ctx_floats) {
    if (d < 1 || !sa_dm(d) || dp < 64 || (dp & 63) || N < 1 || Np < N || (Np & 3) || p < 0.f || !(p < 1.f) ||
        N > (int64_t)1 << 30 || !ctx || ctx_floats < Np * (2 + 3 * (int64_t)sa_dm(d)))
        return U2GNN_E_ARG;
    if (!al16(ctx)) return U2GNN_E_ALIGN;
    return U2GNN_OK;
}

SaP sa_params(int64_t dp, int64_t d, int64_t N, int64_t Np, float p, uint64_t seed, float *ctx) {
    SaP P;
    std::memset(&P, 0, sizeof(P));
    P.dp = (int32_t)dp, P.d = (int32_t)d, P.N = (int32_t)N, P.Np = (int32_t)Np;
    P.p = p, P.seed = seed, P.epoch = u2gnn_cur_epoch(), P.ctx = ctx;
    return P;
}

template <int DM>
int sa_fwd_launch(const SaP &P, hipStream_t st) {
    const int64_t nt = (int64_t)P.Np * 3 * (DM / 4);
    hipLaunchKernelGGL(sa_proj_kernel<DM>, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, st, P);
    hipLaunchKernelGGL((sa_fwd_kernel<DM, false>), dim3((unsigned)((P.Np + SA_RB - 1) / SA_RB)), dim3(SA_NT), 0, st, P,
                       LsP{});
    return u2gnn_launch_status();
}

template <int DM>
int sa_bwd_launch(const SaP &P, hipStream_t st) {
    const dim3 grid((unsigned)((P.Np + SA_RB - 1) / SA_RB));
    hipLaunchKernelGGL((sa_bwd_q_kernel<DM, false>), grid, dim3(SA_NT), 0, st, P, LsP{});
    constexpr int KR = SA_RB * sa_kp<DM>();   // key rows per workgroup
    hipLaunchKernelGGL(sa_bwd_kv_kernel<DM>, dim3((unsigned)((P.Np + KR - 1) / KR)), dim3(SA_NT), 0, st, P);
    return u2gnn_launch_status();
}

}  // namespace

extern "C" {

int64_t u2gnn_attn_small_ctx_floats(int64_t rows_pad, int64_t d) {
    if (!sa_dm(d) || rows_pad < 1) return -1;
    return rows_pad * (2 + 3 * (int64_t)sa_dm(d));
}

int64_t u2gnn_attn_small_ws_floats(int64_t n_valid, int64_t rows_pad, int64_t d) {
    if (!sa_dm(d) || n_valid < 1 || rows_pad < n_valid) return -1;
    return rows_pad * (2 * (int64_t)sa_dm(d) + 4);
}

int u2gnn_attn_small_fwd(const float *X, int64_t ldx, const float *W_in, const float *b_in, int64_t dp, int64_t d,
                         int64_t N, int64_t Np, float p, uint64_t seed, float *O, int64_t ldo, float *ctx,
                         int64_t ctx_floats, void *stream) {
    int rc = sa_check(dp, d, N, Np, p, ctx, ctx_floats);
    if (rc != U2GNN_OK) return rc;
    if (!X || ldx < dp || !W_in || !b_in || !O || ldo < dp) return U2GNN_E_ARG;
    if (!al16(X) || (ldx & 3) || !al16(W_in)) return U2GNN_E_ALIGN;
    SaP P = sa_params(dp, d, N, Np, p, seed, ctx);
    P.x = X, P.ldx = ldx, P.w_in = W_in, P.b_in = b_in, P.q_scale = (float)(1.0 / std::sqrt((double)d));
    P.out = O, P.ld_out = ldo;
    hipStream_t st = u2gnn_stream(stream);
    switch (sa_dm(d)) {
        case 4: return sa_fwd_launch<4>(P, st);
        case 8: return sa_fwd_launch<8>(P, st);
        case 12: return sa_fwd_launch<12>(P, st);
        case 16: return sa_fwd_launch<16>(P, st);
        case 20: return sa_fwd_launch<20>(P, st);
        case 24: return sa_fwd_launch<24>(P, st);
        default: return sa_fwd_launch<32>(P, st);
    }
}

int u2gnn_attn_small_bwd(const float *ctx, int64_t ctx_floats, const float *W_in, int64_t dp, int64_t d, int64_t N,
                         int64_t Np, float p, uint64_t seed, const float *dO, int64_t ld_do, const float *delta,
                         float q_scale, float *dQKV, int64_t ld_dqkv, float *dX, int64_t lddx, float *ws,
                         int64_t ws_floats, void *stream) {
    int rc = sa_check(dp, d, N, Np, p, ctx, ctx_floats);
    if (rc != U2GNN_OK) return rc;
    if (!dO || !delta || !dQKV || ld_dqkv < 3 * dp || ld_do < dp || !ws || ws_floats < u2gnn_attn_small_ws_floats(N, Np, d))
        return U2GNN_E_ARG;
    if (dX && (!W_in || lddx < dp)) return U2GNN_E_ARG;
    if (!al16(dO) || (ld_do & 3) || !al16(ws) || !al16(dQKV) || (ld_dqkv & 3)) return U2GNN_E_ALIGN;
    SaP P = sa_params(dp, d, N, Np, p, seed, const_cast<float *>(ctx));   // read-only in the backward
    P.dO = dO, P.ld_do = ld_do, P.delta = delta, P.q_scale = q_scale;
    P.rq = ws, P.out = dQKV, P.ld_out = ld_dqkv, P.w_in = W_in, P.dx = dX, P.lddx = lddx;
    hipStream_t st = u2gnn_stream(stream);
    switch (sa_dm(d)) {
        case 4: return sa_bwd_launch<4>(P, st);
        case 8: return sa_bwd_launch<8>(P, st);
        case 12: return sa_bwd_launch<12>(P, st);
        case 16: return sa_bwd_launch<16>(P, st);
        case 20: return sa_bwd_launch<20>(P, st);
        case 24: return sa_bwd_launch<24>(P, st);
        default: return sa_bwd_launch<32>(P, st);
    }
}

}  // extern "C"

// ==========================================================================================================
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

namespace {

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
    // every load unconditional from a clamped address, zeroed after (ld4z): the form "zero, then load under a
    // branch" compiled to one s_waitcnt vmcnt(0) per load in the fused kernels (tools/isa_waits.py)
    __device__ __forceinline__ void load(const LsP &P, int h0) {
#pragma unroll
        for (int i = 0; i < P1; ++i) {
            const int e = threadIdx.x + i * LS_NT, h = e / C4, k = 4 * (e % C4);
            a[i] = ld4z(P.a.W1 + (int64_t)min(h0 + h, P.ffp - 1) * P.dp + k, e < N1 && h0 + h < P.ffp);
        }
#pragma unroll
        for (int i = 0; i < P2; ++i) {   // W2 row k, 4 consecutive hidden units (DM rows side by side: their
            // transposed LDS stores below spread over DM x more banks than a row-major walk; 16-way -> 4-way at DM = 4)
            const int e = threadIdx.x + i * LS_NT, k = e % DM, h = 4 * (e / DM);
            b[i] = ld4z(P.a.W2 + (int64_t)k * P.ffp + min(h0 + h, P.ffp - 4), e < N2 && h0 + h < P.ffp);
        }
#pragma unroll
        for (int i = 0; i < P3; ++i) {
            const int e = threadIdx.x + i * LS_NT, h = 4 * e;
            c[i] = ld4z(P.a.b1 + min(h0 + h, P.ffp - 4), e < N3 && h0 + h < P.ffp);
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
            const int e = threadIdx.x + i * LS_NT, k = e % DM, h = 4 * (e / DM);
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
__device__ __forceinline__ float ln_row_v(float z, int lane, int d, float eps, float gam, float bet, float &mu,
                                          float &rs) {   // (gam, bet: column lane's gamma, beta)
    const bool ok = lane < d;
    const float v = ok ? z : 0.f;
    mu = wsum(v) / (float)d;
    const float t = ok ? v - mu : 0.f;
    rs = rsqrtf(wsum(t * t) / (float)d + eps);
    return ok ? t * rs * gam + bet : 0.f;
}
__device__ __forceinline__ float ln_row(float z, int lane, int d, float eps, const float *gamma, const float *beta,
                                        float &mu, float &rs) {
    const int c = lane < d ? lane : 0;   // gamma, beta: unpadded [d]
    return ln_row_v(z, lane, d, eps, gamma[c], beta[c], mu, rs);
}

// LN backward of one row (lane c < d): dz = rs (g - mean(g) - xh mean(g xh)), g = dy gamma, xh = (z - mu) rs
__device__ __forceinline__ float ln_row_bwd_v(float dy, float z, float mu, float rs, int lane, int d, float gam) {
    const bool ok = lane < d;
    const float xh = ok ? (z - mu) * rs : 0.f;
    const float g = ok ? dy * gam : 0.f;
    const float m1 = wsum(g) / (float)d, m2 = wsum(g * xh) / (float)d;
    return ok ? rs * (g - m1 - xh * m2) : 0.f;
}
__device__ __forceinline__ float ln_row_bwd(float dy, float z, float mu, float rs, int lane, int d, const float *gamma) {
    return ln_row_bwd_v(dy, z, mu, rs, lane, d, gamma[lane < d ? lane : 0]);
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
            for (int u = 0; u < NU; ++u) {   // (unconditional loads, clamped: see Stage::load)
                const float v = hrow[min(h0 + 64 * u + lane, P.ffp - 1)];
                hvs[u] = h0 + 64 * u + lane < P.ffp ? v : 0.f;
            }
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

// ---- the tail phase of the fused kernels (sa_fwd_kernel / sa_bwd_q_kernel with TAIL): the workgroup's SA_RB
// rows, SA_SPL waves per row splitting the hidden units of each LDS-staged chunk (unit 64 k + lane, k = sp,
// sp + SA_SPL, ...), the waves' partial sums combined in wave order; the row's finishing wave (sp 0) runs the
// row prologue / epilogue.  Same arithmetic per unit as ls_fwd_kernel / ls_bwd_kernel; the hidden-unit partial
// sums are taken in another order (per wave, then across the two waves).
template <int DM, int SPL> constexpr int tail_smem_floats() {
    return 2 * ls_hc<DM>() * DM + ls_hc<DM>() + SA_WAVES / SPL * (4 * DM + 4);
}

// The tail's global operands are issued ahead of the phase that uses them (round 6, tools/sl_stamps.py: each
// dependent global round trip cost about a microsecond of the workgroup's chain): the row operands (TailRowF /
// TailRowB) at kernel start; forward, the first weight chunk (Stage) right after the walk, under the lane merge,
// the O row and LayerNorm1; backward, the first chunk and the row's ReLU image together with the row operands.
// forward row operands, lane c < d: W_o row c, b_o[c], X[i][c], b2[c], the LayerNorm gammas / betas of column c
template <int DM>
struct TailRowF {
    float wo[DM], bo, x, g1, e1, b2, g2, e2;
    __device__ __forceinline__ void load(const LsP &T, int i) {
        const int lane = threadIdx.x & 63, cw = lane < DM ? lane : 0, c = lane < T.d ? lane : 0;
        const u2gnn_small_tail_args &A = T.a;
#pragma unroll
        for (int k = 0; k < DM; k += 4) {
            const float4 t = *reinterpret_cast<const float4 *>(A.W_o + (int64_t)cw * T.dp + k);
            wo[k] = t.x, wo[k + 1] = t.y, wo[k + 2] = t.z, wo[k + 3] = t.w;
        }
        bo = A.b_o[lane], x = A.X[(int64_t)i * T.dp + lane], b2 = A.b2[lane];   // (dp == 64: one column per lane)
        g1 = A.n1_w[c], e1 = A.n1_b[c], g2 = A.n2_w[c], e2 = A.n2_b[c];
    }
};

// backward row operands, lane c: dX2, Z2, Z1, O of column c, the row statistics, the LayerNorm gammas, W_o column c
template <int DM>
struct TailRowB {
    float dx2, z2, mu2, rs2, g2, z1, mu1, rs1, g1, o, woc[DM];
    __device__ __forceinline__ void load(const LsP &T, int i) {
        const int lane = threadIdx.x & 63, kc = lane < DM ? lane : 0, c = lane < T.d ? lane : 0;
        const u2gnn_small_tail_args &A = T.a;
        const int64_t ro = (int64_t)i * T.dp;
        dx2 = A.dX2[ro + lane], z2 = A.Z2[ro + lane], z1 = A.Z1[ro + lane], o = A.O[ro + lane];
        mu2 = A.mean2[i], rs2 = A.rstd2[i], mu1 = A.mean1[i], rs1 = A.rstd1[i];
        g2 = A.n2_w[c], g1 = A.n1_w[c];
#pragma unroll
        for (int k = 0; k < DM; ++k) woc[k] = A.W_o[(int64_t)k * T.dp + kc];
    }
};

// the row's ReLU image Hd over this wave's units of chunk h0
template <int DM, int SPL>
__device__ void tail_hd_load(const LsP &T, int i, int sp, int h0, float (&hvs)[ls_nw<DM, SPL>()]) {
    constexpr int NU = ls_hc<DM>() / 64;
    const int lane = threadIdx.x & 63;
    const float *hrow = T.a.Hd + (int64_t)i * T.ffp;
    // every load issued unconditionally (clamped index, masked after): a conditional load into a zeroed register
    // compiled to load -> s_waitcnt vmcnt(0) per unit, a memory round trip each (tools/isa_waits.py)
    float v[ls_nw<DM, SPL>()];
#pragma unroll
    for (int u = 0; u < ls_nw<DM, SPL>(); ++u) {
        const int k = sp + SPL * u, h = 64 * k + lane;
        v[u] = hrow[min(h0 + h, T.ffp - 1)];
    }
#pragma unroll
    for (int u = 0; u < ls_nw<DM, SPL>(); ++u) {
        const int k = sp + SPL * u, h = 64 * k + lane;
        hvs[u] = (k < NU && h0 + h < T.ffp) ? v[u] : 0.f;
    }
}

template <int DM, int SPL>
__device__ void tail_fwd_rows(const LsP &T, int i, int rw, int sp, const float (&of)[DM], bool fin,
                              const TailRowF<DM> &rp, Stage<DM, ls_hc<DM>(), true> &sg, float *smem) {
    static_assert(LS_NT == SA_NT, "the tail's staging runs on the attention workgroup");
    constexpr int RB = SA_WAVES / SPL;
    constexpr int HC = ls_hc<DM>(), NPR = (HC / 2 + 63) / 64;   // 64-lane rounds of unit pairs per chunk
    float (*w1s)[DM] = reinterpret_cast<float (*)[DM]>(smem);
    float (*w2s)[DM] = reinterpret_cast<float (*)[DM]>(smem + HC * DM);
    float *b1s = smem + 2 * HC * DM;
    float (*xs)[DM] = reinterpret_cast<float (*)[DM]>(b1s + HC);
    float (*xz)[SPL][DM] = reinterpret_cast<float (*)[SPL][DM]>(b1s + HC + RB * DM);
    const int lane = threadIdx.x & 63;
    const bool live = i < T.N;
    const u2gnn_small_tail_args &A = T.a;
    const bool drop = T.p > 0.f;
    const float ks = drop ? 1.f / (1.f - T.p) : 1.f;
    const uint32_t thr = u2gnn_keep_thr(T.p);
    const uint64_t s1 = u2gnn_seed(T.s1, T.epoch), sff = u2gnn_seed(T.sff, T.epoch), s2 = u2gnn_seed(T.s2, T.epoch);
    const int64_t ro = (int64_t)i * T.dp;
    // a3.3 from the O row in registers: z1 = drop1(O W_o^T + b_o) + x, LayerNorm1
    float x1 = 0.f;
    if (fin) {
        float z1 = 0.f, mu1 = 0.f, rs1 = 0.f;
        if (live) {
            float acc = 0.f;
#pragma unroll
            for (int k = 0; k < DM; ++k) acc = fmaf(of[k], rp.wo[k], acc);
            float v = acc + rp.bo;
            if (drop) v = u2gnn_keep(s1, (uint32_t)i, (uint32_t)lane, T.p) ? v * ks : 0.f;
            z1 = lane < T.d ? v + rp.x : 0.f;
            x1 = ln_row_v(z1, lane, T.d, T.eps, rp.g1, rp.e1, mu1, rs1);
        }
        A.Z1[ro + lane] = z1;
        A.X1[ro + lane] = x1;
        if (lane == 0) A.mean1[i] = mu1, A.rstd1[i] = rs1;
        if (lane < DM) xs[rw][lane] = x1;
    }
    __syncthreads();
    SX_STAMP(0, 5);
    float xv[DM], zp[DM];
#pragma unroll
    for (int k = 0; k < DM; ++k) xv[k] = xs[rw][k], zp[k] = 0.f;
    // a3.4 over this wave's hidden units
    const uint32_t rkf = u2gnn_row_key(sff, (uint32_t)i);
    float *hrow = A.Hd + (int64_t)i * T.ffp;
    for (int h0 = 0; h0 < T.ffp; h0 += HC) {
        if (h0) __syncthreads();   // the previous chunk's readers are done
        sg.store(w1s, w2s, b1s);
        __syncthreads();
        if (h0 + HC < T.ffp) sg.load(T, h0 + HC);   // the next chunk, in flight under this one
        if (h0 == 0) SX_STAMP(0, 6);
        // unit pairs (h, h + 1), h = 2 (64 k + lane): one dropout hash per pair gives both keep bits, Hd written as
        // float2 (round 6: a hash per unit was a fifth of the kernel's VALU issue)
#pragma unroll 2
        for (int k = sp; k < NPR; k += SPL) {
            const int h = 2 * (64 * k + lane);
            if (h >= HC || h0 + h >= T.ffp) break;   // (ffp even: h + 1 < ffp too)
            float a0 = b1s[h], a1 = b1s[h + 1];
#pragma unroll
            for (int c = 0; c < DM; c += 4) {
                const float4 t0 = *reinterpret_cast<const float4 *>(&w1s[h][c]);
                const float4 t1 = *reinterpret_cast<const float4 *>(&w1s[h + 1][c]);
                a0 = fmaf(xv[c], t0.x, a0), a0 = fmaf(xv[c + 1], t0.y, a0), a0 = fmaf(xv[c + 2], t0.z, a0);
                a0 = fmaf(xv[c + 3], t0.w, a0);
                a1 = fmaf(xv[c], t1.x, a1), a1 = fmaf(xv[c + 1], t1.y, a1), a1 = fmaf(xv[c + 2], t1.z, a1);
                a1 = fmaf(xv[c + 3], t1.w, a1);
            }
            bool k0 = true, k1 = true;
            if (drop) {
                const uint32_t hh = u2gnn_pair_hash(rkf, (uint32_t)(h0 + h) >> 1);
                k0 = u2gnn_keep_lo(hh, thr), k1 = u2gnn_keep_hi(hh, thr);
            }
            a0 = (live && k0) ? fmaxf(a0, 0.f) * ks : 0.f;
            a1 = (live && k1) ? fmaxf(a1, 0.f) * ks : 0.f;
            *reinterpret_cast<float2 *>(hrow + h0 + h) = make_float2(a0, a1);
#pragma unroll
            for (int c = 0; c < DM; c += 4) {
                const float4 q0 = *reinterpret_cast<const float4 *>(&w2s[h][c]);
                const float4 q1 = *reinterpret_cast<const float4 *>(&w2s[h + 1][c]);
                zp[c] = fmaf(a1, q1.x, fmaf(a0, q0.x, zp[c]));
                zp[c + 1] = fmaf(a1, q1.y, fmaf(a0, q0.y, zp[c + 1]));
                zp[c + 2] = fmaf(a1, q1.z, fmaf(a0, q0.z, zp[c + 2]));
                zp[c + 3] = fmaf(a1, q1.w, fmaf(a0, q0.w, zp[c + 3]));
            }
        }
    }
    SX_STAMP(0, 7);
#pragma unroll
    for (int k = 0; k < DM; ++k) zp[k] = wsum(zp[k]);
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < DM; ++k) xz[rw][sp][k] = zp[k];
    __syncthreads();
    SX_STAMP(0, 8);
    if (!fin) return;
#pragma unroll
    for (int k = 0; k < DM; ++k) {
        float t = xz[rw][0][k];
#pragma unroll
        for (int y = 1; y < SPL; ++y) t += xz[rw][y][k];
        zp[k] = t;
    }
    float z2 = 0.f, x2 = 0.f, mu2 = 0.f, rs2 = 0.f;
    if (live) {
        float v = pick<DM>(zp, lane) + rp.b2;
        if (drop) v = u2gnn_keep(s2, (uint32_t)i, (uint32_t)lane, T.p) ? v * ks : 0.f;
        z2 = lane < T.d ? v + x1 : 0.f;
        x2 = ln_row_v(z2, lane, T.d, T.eps, rp.g2, rp.e2, mu2, rs2);
    }
    A.Z2[ro + lane] = z2;
    A.X2[ro + lane] = x2;
    if (lane == 0) A.mean2[i] = mu2, A.rstd2[i] = rs2;
}

// the tail backward of the row; on return every wave of the row holds its dO row (g) and delta (dl).  sg, hvs: the
// first chunk's weights and this wave's units of the row's ReLU image, already in flight
template <int DM, int SPL>
__device__ void tail_bwd_rows(const LsP &T, int i, int rw, int sp, bool fin, const TailRowB<DM> &rp,
                              Stage<DM, ls_hc<DM>(), false> &sg, float (&hvs)[ls_nw<DM, SPL>()], float (&g)[DM], float &dl,
                              float *smem) {
    constexpr int HC = ls_hc<DM>(), NU = HC / 64, NW = ls_nw<DM, SPL>(), RB = SA_WAVES / SPL;
    float (*w1s)[DM] = reinterpret_cast<float (*)[DM]>(smem);
    float (*w2s)[DM] = reinterpret_cast<float (*)[DM]>(smem + HC * DM);
    float (*fs)[DM] = reinterpret_cast<float (*)[DM]>(smem + 2 * HC * DM);
    float (*xz)[SPL][DM] = reinterpret_cast<float (*)[SPL][DM]>(smem + 2 * HC * DM + RB * DM);
    float (*gs)[DM + 4] = reinterpret_cast<float (*)[DM + 4]>(smem + 2 * HC * DM + RB * DM * (1 + SPL));
    const int lane = threadIdx.x & 63;
    const bool live = i < T.N;
    const u2gnn_small_tail_args &A = T.a;
    const bool drop = T.p > 0.f;
    const float ks = drop ? 1.f / (1.f - T.p) : 1.f;
    const uint64_t s1 = u2gnn_seed(T.s1, T.epoch), s2 = u2gnn_seed(T.s2, T.epoch);
    const int64_t ro = (int64_t)i * T.dp;
    // LayerNorm2^T -> dz2 (kept by the finishing wave), dF
    float dz2 = 0.f;
    if (fin) {
        float df = 0.f;
        if (live) {
            dz2 = ln_row_bwd_v(rp.dx2, rp.z2, rp.mu2, rp.rs2, lane, T.d, rp.g2);
            df = (drop && lane < T.d) ? (u2gnn_keep(s2, (uint32_t)i, (uint32_t)lane, T.p) ? dz2 * ks : 0.f) : dz2;
        }
        A.dF[ro + lane] = df;
        if (lane < DM) fs[rw][lane] = df;
    }
    __syncthreads();
    SX_STAMP(1, 5);
    float fv[DM], xp[DM];
#pragma unroll
    for (int k = 0; k < DM; ++k) fv[k] = fs[rw][k], xp[k] = 0.f;
    float *dhrow = A.dH + (int64_t)i * T.ffp;
    for (int h0 = 0; h0 < T.ffp; h0 += HC) {
        if (h0) __syncthreads();   // the previous chunk's readers are done
        sg.store(w1s, w2s, nullptr);
        __syncthreads();
        float hc[NW];
#pragma unroll
        for (int u = 0; u < NW; ++u) hc[u] = hvs[u];
        if (h0 + HC < T.ffp) {   // the next chunk, in flight under this one
            sg.load(T, h0 + HC);
            tail_hd_load<DM, SPL>(T, i, sp, h0 + HC, hvs);
        }
        if (h0 == 0) SX_STAMP(1, 6);
#pragma unroll 4
        for (int u = 0; u < NW; ++u) {
            const int k = sp + SPL * u, h = 64 * k + lane;
            if (k >= NU || h0 + h >= T.ffp) break;
            float w1[DM], w2[DM];
#pragma unroll
            for (int c = 0; c < DM; c += 4) {
                const float4 t = *reinterpret_cast<const float4 *>(&w1s[h][c]);
                w1[c] = t.x, w1[c + 1] = t.y, w1[c + 2] = t.z, w1[c + 3] = t.w;
                const float4 q = *reinterpret_cast<const float4 *>(&w2s[h][c]);
                w2[c] = q.x, w2[c + 1] = q.y, w2[c + 2] = q.z, w2[c + 3] = q.w;
            }
            ffn_unit_bwd<DM>(fv, w1, w2, hc[u], ks, live, dhrow + h0 + h, xp);
        }
    }
    SX_STAMP(1, 7);
#pragma unroll
    for (int k = 0; k < DM; ++k) xp[k] = wsum(xp[k]);
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < DM; ++k) xz[rw][sp][k] = xp[k];
    __syncthreads();
    SX_STAMP(1, 8);
    if (fin) {
#pragma unroll
        for (int k = 0; k < DM; ++k) {
            float t = xz[rw][0][k];
#pragma unroll
            for (int y = 1; y < SPL; ++y) t += xz[rw][y][k];
            xp[k] = t;
        }
        float dx1 = 0.f, dz1 = 0.f, da = 0.f, dov = 0.f, dlt = 0.f;
        if (live) {
            dx1 = lane < T.d ? dz2 + pick<DM>(xp, lane) : 0.f;
            dz1 = ln_row_bwd_v(dx1, rp.z1, rp.mu1, rp.rs1, lane, T.d, rp.g1);
            da = (drop && lane < T.d) ? (u2gnn_keep(s1, (uint32_t)i, (uint32_t)lane, T.p) ? dz1 * ks : 0.f) : dz1;
            float av[DM];
#pragma unroll
            for (int k = 0; k < DM; ++k) av[k] = __shfl(da, k, 64);
            float acc = 0.f;
#pragma unroll
            for (int c = 0; c < DM; ++c) acc = fmaf(av[c], rp.woc[c], acc);
            dov = lane < T.d ? acc : 0.f;
            dlt = wsum(dov * rp.o);
        }
        A.dX1[ro + lane] = dx1;
        A.dX[ro + lane] = dz1;
        A.dA[ro + lane] = da;
        A.dO[ro + lane] = dov;
        if (lane == 0) A.delta[i] = dlt, gs[rw][DM] = dlt;
        if (lane < DM) gs[rw][lane] = dov;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < DM; ++k) g[k] = gs[rw][k];
    dl = gs[rw][DM];
}

int ls_dm(int64_t d) { return d < 1 ? 0 : d <= 24 ? (int)((d + 3) / 4 * 4) : d <= 32 ? 32 : 0; }

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
    P.s1 = a->seed_drop1, P.sff = a->seed_dropff, P.s2 = a->seed_drop2, P.epoch = u2gnn_cur_epoch();
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

// ---- a whole small-width layer (ABI u2gnn_layer_small_fwd / _bwd): fused where the rows allow --------------
// rows_pad >= 1024 (the tail's STAGED split): attention forward + tail in one launch, tail backward + the dQ walk
// in one launch; below that the tail's DIRECT split keeps its own launches
#ifndef SMALL_FUSE_ROWS_
#define SMALL_FUSE_ROWS_ 1024
#endif
constexpr int64_t SMALL_FUSE_ROWS = SMALL_FUSE_ROWS_;   // (C5: fused 0.541 / 0.543 vs separate 0.587 / 0.594 ms, one session)

template <int DM>
int small_fwd_launch(const SaP &P, const LsP &T, hipStream_t st) {
    const int64_t nt = (int64_t)P.Np * 3 * (DM / 4);
    hipLaunchKernelGGL(sa_proj_kernel<DM>, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, st, P);
    const dim3 grid((unsigned)((P.Np + SA_RB - 1) / SA_RB));
    if (P.Np >= SMALL_FUSE_ROWS) {   // (DM = 4: one wave per row, SA_FWD_SPL; wider rows spill registers there)
        constexpr int FS = DM <= 4 ? SA_FWD_SPL : SA_SPL, RBF = SA_WAVES / FS;
        hipLaunchKernelGGL((sa_fwd_kernel<DM, true, FS>), dim3((unsigned)((P.Np + RBF - 1) / RBF)), dim3(SA_NT), 0, st, P,
                           T);
    } else {
        hipLaunchKernelGGL((sa_fwd_kernel<DM, false>), grid, dim3(SA_NT), 0, st, P, LsP{});
        hipLaunchKernelGGL((ls_fwd_kernel<DM, true>), dim3((unsigned)P.Np), dim3(LS_NT), 0, st, T);
    }
    return u2gnn_launch_status();
}

template <int DM>
int small_bwd_launch(const SaP &P, const LsP &T, hipStream_t st) {
    const dim3 grid((unsigned)((P.Np + SA_RB - 1) / SA_RB));
    if (P.Np >= SMALL_FUSE_ROWS) {
        constexpr int BS = DM <= 4 ? SA_BWD_SPL : SA_SPL, RBB = SA_WAVES / BS;
        hipLaunchKernelGGL((sa_bwd_q_kernel<DM, true, BS>), dim3((unsigned)((P.Np + RBB - 1) / RBB)), dim3(SA_NT), 0, st,
                           P, T);
    } else {
        hipLaunchKernelGGL((ls_bwd_kernel<DM, true>), dim3((unsigned)P.Np), dim3(LS_NT), 0, st, T);
        hipLaunchKernelGGL((sa_bwd_q_kernel<DM, false>), grid, dim3(SA_NT), 0, st, P, LsP{});
    }
    constexpr int KR = SA_RB * sa_kp<DM>();
    hipLaunchKernelGGL(sa_bwd_kv_kernel<DM>, dim3((unsigned)((P.Np + KR - 1) / KR)), dim3(SA_NT), 0, st, P);
    return u2gnn_launch_status();
}

}  // namespace

extern "C" {

#ifdef SX_STAMPS
int u2gnn_dbg_sx_stamps(unsigned long long *host, int64_t n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_sx_stamps), (size_t)n * 8) == hipSuccess ? U2GNN_OK : U2GNN_E_ARG;
}
#endif

int u2gnn_layer_tail_small_fwd(const u2gnn_small_tail_args *a, void *stream) { return ls_run(a, false, stream); }

int u2gnn_layer_tail_small_bwd(const u2gnn_small_tail_args *a, void *stream) { return ls_run(a, true, stream); }


int u2gnn_layer_small_fwd(const u2gnn_small_tail_args *t, const float *W_in, const float *b_in, uint64_t attn_seed,
                          float *ctx, int64_t ctx_floats, void *stream) {
    int rc = ls_check(t, false);
    if (rc != U2GNN_OK) return rc;
    rc = sa_check(t->dp, t->d, t->n_valid, t->rows_pad, t->p, ctx, ctx_floats);
    if (rc != U2GNN_OK) return rc;
    if (!W_in || !b_in) return U2GNN_E_ARG;
    if (!al16(t->X) || !al16(W_in)) return U2GNN_E_ALIGN;
    SaP P = sa_params(t->dp, t->d, t->n_valid, t->rows_pad, t->p, attn_seed, ctx);
    P.x = t->X, P.ldx = t->dp, P.w_in = W_in, P.b_in = b_in, P.q_scale = (float)(1.0 / std::sqrt((double)t->d));
    P.out = const_cast<float *>(t->O), P.ld_out = t->dp;   // (the attention output: written here)
    const LsP T = ls_params(t);
    hipStream_t st = u2gnn_stream(stream);
    switch (sa_dm(t->d)) {
        case 4: return small_fwd_launch<4>(P, T, st);
        case 8: return small_fwd_launch<8>(P, T, st);
        case 12: return small_fwd_launch<12>(P, T, st);
        case 16: return small_fwd_launch<16>(P, T, st);
        case 20: return small_fwd_launch<20>(P, T, st);
        case 24: return small_fwd_launch<24>(P, T, st);
        default: return small_fwd_launch<32>(P, T, st);
    }
}

int u2gnn_layer_small_bwd(const u2gnn_small_tail_args *t, const float *W_in, uint64_t attn_seed, const float *ctx,
                          int64_t ctx_floats, float *dQKV, int64_t ld_dqkv, int32_t accumulate_dx, float *ws,
                          int64_t ws_floats, void *stream) {
    int rc = ls_check(t, true);
    if (rc != U2GNN_OK) return rc;
    rc = sa_check(t->dp, t->d, t->n_valid, t->rows_pad, t->p, ctx, ctx_floats);
    if (rc != U2GNN_OK) return rc;
    if (!dQKV || ld_dqkv < 3 * t->dp || !ws || ws_floats < u2gnn_attn_small_ws_floats(t->n_valid, t->rows_pad, t->d) ||
        (accumulate_dx && !W_in))
        return U2GNN_E_ARG;
    if (!al16(ws) || !al16(dQKV) || (ld_dqkv & 3) || !al16(t->dO)) return U2GNN_E_ALIGN;
    SaP P = sa_params(t->dp, t->d, t->n_valid, t->rows_pad, t->p, attn_seed, const_cast<float *>(ctx));
    P.dO = t->dO, P.ld_do = t->dp, P.delta = t->delta, P.q_scale = (float)(1.0 / std::sqrt((double)t->d));
    P.rq = ws, P.out = dQKV, P.ld_out = ld_dqkv, P.w_in = W_in;
    P.dx = accumulate_dx ? t->dX : nullptr, P.lddx = t->dp;
    const LsP T = ls_params(t);
    hipStream_t st = u2gnn_stream(stream);
    switch (sa_dm(t->d)) {
        case 4: return small_bwd_launch<4>(P, T, st);
        case 8: return small_bwd_launch<8>(P, T, st);
        case 12: return small_bwd_launch<12>(P, T, st);
        case 16: return small_bwd_launch<16>(P, T, st);
        case 20: return small_bwd_launch<20>(P, T, st);
        case 24: return small_bwd_launch<24>(P, T, st);
        default: return small_bwd_launch<32>(P, T, st);
    }
}

}  // extern "C"
