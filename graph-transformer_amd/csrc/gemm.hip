// Dense contractions of the U2GNN encoder on gfx950 matrix cores.
//
// Replaces the ATen GEMMs the reference reaches through torch.nn.TransformerEncoderLayer
// (pytorch_U2GNN_Sup.py:19-21,35 / pytorch_U2GNN_UnSup.py:37-40,57): the MHA in-projection,
// Q.K^T, P.V, the out-projection, the two FFN linears, and every product of their backward.
//
// Design (gfx950):
//   * 256-thread workgroups = 4 wave64s in a 2x2 arrangement; each wave owns a
//     (BM/2)x(BN/2) output tile made of 32x32 MFMA tiles, accumulators in registers.
//   * fp32 path: v_mfma_f32_32x32x2_f32 — exact fp32 fma chains (the reference computes in
//     fp32; this is the parity-grade path).  Operands staged through LDS k-major
//     ([BK][BM+pad]) so each MFMA operand is one conflict-free ds_read_b32 per lane.
//   * global->LDS by register staging with float4 loads (16 B/lane, coalesced along the
//     contiguous dimension of either layout), two LDS buffers, one barrier per K tile, the
//     next tile's loads in flight under the current tile's MFMAs.
//   * bijective XCD-aware block remap (blocks b, b+8 share an XCD) + grouped tile order so
//     the 8 private L2s each see a compact set of A row-panels and B column-panels.
//   * fused epilogues (bias, q-scaling, relu, dropout, residual, attention dS) so no
//     elementwise pass re-reads a GEMM output.
//   * split-K writes fp32 partial slabs (deterministic; reduced by u2gnn_slab_reduce).
#include "u2gnn_common.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

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
};

template <int EPI>
__device__ __forceinline__ float epilogue(const GemmP &P, int row, int col, float acc) {
    if constexpr (EPI == U2GNN_EPI_STORE) {
        return P.alpha * acc;
    } else if constexpr (EPI == U2GNN_EPI_BIAS) {
        float v = acc + P.bias[col];
        return col < P.scale_cols ? v * P.alpha : v;
    } else if constexpr (EPI == U2GNN_EPI_BIAS_DROP_RESID) {
        float v = acc + P.bias[col];
        if (P.p > 0.f) v = u2gnn_keep(P.seed, row, col, P.p) ? v * (1.f / (1.f - P.p)) : 0.f;
        return P.aux0[(int64_t)row * P.ld_aux + col] + v;
    } else if constexpr (EPI == U2GNN_EPI_BIAS_RELU_DROP) {
        float v = fmaxf(acc + P.bias[col], 0.f);
        if (P.p > 0.f) v = u2gnn_keep(P.seed, row, col, P.p) ? v * (1.f / (1.f - P.p)) : 0.f;
        return v;
    } else if constexpr (EPI == U2GNN_EPI_RELU_DROP_BWD) {
        const float h = P.aux0[(int64_t)row * P.ld_aux + col];
        return h > 0.f ? acc * (1.f / (1.f - P.p)) : 0.f;
    } else if constexpr (EPI == U2GNN_EPI_ACCUM) {
        return P.C[(int64_t)row * P.ldc + col] + P.alpha * acc;
    } else {  // U2GNN_EPI_ATTN_DS
        const int64_t o = (int64_t)row * P.ld_aux + col;
        return P.aux1[o] * acc - P.aux0[o] * P.rowvec[row];
    }
}

__device__ __forceinline__ void tile_coords(int gm, int gn, int &tm, int &tn) {
    const int nwg = gm * gn;
    const int bid = blockIdx.x;
    const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7, loc = bid >> 3;
    const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
    constexpr int GROUP = 8;
    const int per_group = GROUP * gn;
    const int g = wgid / per_group;
    const int first_m = g * GROUP;
    const int gsz = min(gm - first_m, GROUP);
    const int in_g = wgid - g * per_group;
    tm = first_m + in_g % gsz;
    tn = in_g / gsz;
}


template <int BM, int BN, int BK, bool TA, bool TB>
__device__ __forceinline__ void g2r(const float *Ab, const float *Bb, int64_t lda, int64_t ldb, int kt,
                                    int tid, float4 (&ra)[BM * BK / 1024], float4 (&rb)[BN * BK / 1024]) {
    constexpr int NA = BM * BK / 1024, NB = BN * BK / 1024;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
        const int idx = tid + i * 256;
        if constexpr (!TA) {
            const int r = idx / (BK / 4), kq = idx % (BK / 4);
            ra[i] = *reinterpret_cast<const float4 *>(Ab + (int64_t)r * lda + kt * BK + kq * 4);
        } else {
            const int k = idx / (BM / 4), mq = idx % (BM / 4);
            ra[i] = *reinterpret_cast<const float4 *>(Ab + (int64_t)(kt * BK + k) * lda + mq * 4);
        }
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const int idx = tid + i * 256;
        if constexpr (TB) {
            const int r = idx / (BK / 4), kq = idx % (BK / 4);
            rb[i] = *reinterpret_cast<const float4 *>(Bb + (int64_t)r * ldb + kt * BK + kq * 4);
        } else {
            const int k = idx / (BN / 4), nq = idx % (BN / 4);
            rb[i] = *reinterpret_cast<const float4 *>(Bb + (int64_t)(kt * BK + k) * ldb + nq * 4);
        }
    }
}

template <int BM, int BN, int BK, int SA, int SB, bool TA, bool TB>
__device__ __forceinline__ void r2s(float *As, float *Bs, int tid, const float4 (&ra)[BM * BK / 1024],
                                    const float4 (&rb)[BN * BK / 1024]) {
    constexpr int NA = BM * BK / 1024, NB = BN * BK / 1024;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
        const int idx = tid + i * 256;
        if constexpr (!TA) {
            const int r = idx / (BK / 4), kq = idx % (BK / 4);
            As[(kq * 4 + 0) * SA + r] = ra[i].x;
            As[(kq * 4 + 1) * SA + r] = ra[i].y;
            As[(kq * 4 + 2) * SA + r] = ra[i].z;
            As[(kq * 4 + 3) * SA + r] = ra[i].w;
        } else {
            const int k = idx / (BM / 4), mq = idx % (BM / 4);
            *reinterpret_cast<float4 *>(As + k * SA + mq * 4) = ra[i];
        }
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const int idx = tid + i * 256;
        if constexpr (TB) {
            const int r = idx / (BK / 4), kq = idx % (BK / 4);
            Bs[(kq * 4 + 0) * SB + r] = rb[i].x;
            Bs[(kq * 4 + 1) * SB + r] = rb[i].y;
            Bs[(kq * 4 + 2) * SB + r] = rb[i].z;
            Bs[(kq * 4 + 3) * SB + r] = rb[i].w;
        } else {
            const int k = idx / (BN / 4), nq = idx % (BN / 4);
            *reinterpret_cast<float4 *>(Bs + k * SB + nq * 4) = rb[i];
        }
    }
}

// ------------------------------------------------------------------------------------
// fp32 MFMA kernel
// ------------------------------------------------------------------------------------
template <int BM, int BN, bool TA, bool TB, int EPI>
__global__ void __launch_bounds__(256) gemm_f32_kernel(GemmP P) {
    constexpr int BK = 16;
    constexpr int WTM = BM / 2, WTN = BN / 2;
    constexpr int TM = WTM / 32, TN = WTN / 32;
    constexpr int SA = BM + (TA ? 4 : 2);
    constexpr int SB = BN + (TB ? 2 : 4);
    constexpr int NA = BM * BK / 4 / 256;
    constexpr int NB = BN * BK / 4 / 256;
    static_assert(NA >= 1 && NB >= 1, "tile too small for 256 threads");
    __shared__ __attribute__((aligned(16))) float smem[2 * BK * (SA + SB)];
    float *As0 = smem;
    float *Bs0 = smem + 2 * BK * SA;

    const int tid = threadIdx.x;
    int tmi, tni;
    tile_coords(P.gm, P.gn, tmi, tni);
    const int m0 = tmi * BM, n0 = tni * BN;
    const int64_t kbase = (int64_t)blockIdx.z * P.K;

    const float *Ab = TA ? P.A + kbase * P.lda + m0 : P.A + (int64_t)m0 * P.lda + kbase;
    const float *Bb = TB ? P.B + (int64_t)n0 * P.ldb + kbase : P.B + kbase * P.ldb + n0;

    float4 ra[NA], rb[NB];
    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int wave = tid >> 6, lane = tid & 63;
    const int wm = wave >> 1, wn = wave & 1;
    const int kh = lane >> 5, li = lane & 31;
    const int64_t klen = min((int64_t)P.K, (int64_t)P.Ktot - kbase);
    const int nk = klen > 0 ? (int)(klen / BK) : 0;   // ragged last split; empty splits write 0

    if (nk > 0) {
        g2r<BM, BN, BK, TA, TB>(Ab, Bb, P.lda, P.ldb, 0, tid, ra, rb);
        r2s<BM, BN, BK, SA, SB, TA, TB>(As0, Bs0, tid, ra, rb);
        __syncthreads();
    }
    for (int t = 0; t < nk; ++t) {
        // unconditional prefetch (the last iteration re-reads the final tile; harmless) keeps
        // the staging registers out of scratch
        g2r<BM, BN, BK, TA, TB>(Ab, Bb, P.lda, P.ldb, min(t + 1, nk - 1), tid, ra, rb);
        const float *as = As0 + (t & 1) * BK * SA + wm * WTM + li;
        const float *bs = Bs0 + (t & 1) * BK * SB + wn * WTN + li;
#pragma unroll
        for (int kk = 0; kk < BK / 2; ++kk) {
            const int k = 2 * kk + kh;
            float a[TM], b[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) a[i] = as[k * SA + i * 32];
#pragma unroll
            for (int j = 0; j < TN; ++j) b[j] = bs[k * SB + j * 32];
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
        }
        r2s<BM, BN, BK, SA, SB, TA, TB>(As0 + ((t + 1) & 1) * BK * SA, Bs0 + ((t + 1) & 1) * BK * SB, tid, ra, rb);
        __syncthreads();
    }

    float *C = P.C + (int64_t)blockIdx.z * P.slab_stride;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = m0 + wm * WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * kh;
                const int col = n0 + wn * WTN + j * 32 + li;
                C[(int64_t)row * P.ldc + col] = epilogue<EPI>(P, row, col, acc[i][j][r]);
            }
}

// ------------------------------------------------------------------------------------
// split-bf16 MFMA kernel (U2GNN_PREC_BF16X3) and plain bf16 (U2GNN_PREC_BF16)
//
// x = hi + lo with hi = bf16(x), lo = bf16(x - hi) (|x - hi - lo| <= 2^-17 |x|); the product is
// hi*hi + hi*lo + lo*hi on v_mfma_f32_32x32x16_bf16 with fp32 accumulation, i.e. ~2^-16
// relative error per product at 3 bf16 MFMAs (5.3x the fp32-MFMA rate).  fp32 operands are
// split once per block while staging into LDS (register staging; the split is VALU work that
// runs beside the matrix pipe), so HBM/L2 traffic is the fp32 operands themselves.
// LDS holds both operands k-contiguous ([rows][BK+8] bf16: 80-byte rows make the
// ds_read_b128 fragment reads conflict-free); [K][rows] layouts are transposed in registers
// (4k x 4m micro-tiles) on the way in.
// ------------------------------------------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

template <int R, int BK, bool T>
__device__ __forceinline__ void g2r_bf(const float *base, int64_t ld, int kt, int tid, float4 (&v)[R * BK / 1024]) {
    constexpr int NF = R * BK / 1024;
    if constexpr (!T) {  // global [R][K]
#pragma unroll
        for (int i = 0; i < NF; ++i) {
            const int idx = tid + i * 256;
            const int r = idx / (BK / 4), kq = idx % (BK / 4);
            v[i] = *reinterpret_cast<const float4 *>(base + (int64_t)r * ld + kt * BK + kq * 4);
        }
    } else {  // global [K][R]: NF k-rows x 4 columns per thread
        const int mg = tid % (R / 4), kg = tid / (R / 4);
#pragma unroll
        for (int q = 0; q < NF; ++q)
            v[q] = *reinterpret_cast<const float4 *>(base + (int64_t)(kt * BK + kg * NF + q) * ld + mg * 4);
    }
}

template <int R, int BK, int LDK, bool T, bool SPLIT>
__device__ __forceinline__ void r2s_bf(__bf16 *hi, __bf16 *lo, int tid, const float4 (&v)[R * BK / 1024]) {
    constexpr int NF = R * BK / 1024;
    if constexpr (!T) {
#pragma unroll
        for (int i = 0; i < NF; ++i) {
            const int idx = tid + i * 256;
            const int r = idx / (BK / 4), kq = idx % (BK / 4);
            const float x[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
            bf16x4 h, l;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                h[c] = (__bf16)x[c];
                l[c] = (__bf16)(x[c] - (float)h[c]);
            }
            *reinterpret_cast<bf16x4 *>(hi + r * LDK + kq * 4) = h;
            if constexpr (SPLIT) *reinterpret_cast<bf16x4 *>(lo + r * LDK + kq * 4) = l;
        }
    } else {
        const int mg = tid % (R / 4), kg = tid / (R / 4);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            float x[NF];
#pragma unroll
            for (int q = 0; q < NF; ++q) x[q] = c == 0 ? v[q].x : c == 1 ? v[q].y : c == 2 ? v[q].z : v[q].w;
            __bf16 *dh = hi + (mg * 4 + c) * LDK + kg * NF;
            __bf16 *dl = lo + (mg * 4 + c) * LDK + kg * NF;
            if constexpr (NF == 4) {
                bf16x4 h, l;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    h[q] = (__bf16)x[q];
                    l[q] = (__bf16)(x[q] - (float)h[q]);
                }
                *reinterpret_cast<bf16x4 *>(dh) = h;
                if constexpr (SPLIT) *reinterpret_cast<bf16x4 *>(dl) = l;
            } else {
                static_assert(NF == 2, "bf16 staging supports 64- and 128-row tiles");
                bf16x2 h, l;
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    h[q] = (__bf16)x[q];
                    l[q] = (__bf16)(x[q] - (float)h[q]);
                }
                *reinterpret_cast<bf16x2 *>(dh) = h;
                if constexpr (SPLIT) *reinterpret_cast<bf16x2 *>(dl) = l;
            }
        }
    }
}

template <int BM, int BN, bool TA, bool TB, int EPI, bool SPLIT>
__global__ void __launch_bounds__(256) gemm_bf16_kernel(GemmP P) {
    constexpr int BK = 32;
    constexpr int LDK = BK + 8;
    constexpr int WTM = BM / 2, WTN = BN / 2;
    constexpr int TM = WTM / 32, TN = WTN / 32;
    constexpr int NFA = BM * BK / 1024, NFB = BN * BK / 1024;
    constexpr int AE = BM * LDK, BE = BN * LDK;
    constexpr int STAGE = 2 * (AE + BE);  // hi + lo of A and B
    __shared__ __attribute__((aligned(16))) __bf16 smem[2 * STAGE];

    const int tid = threadIdx.x;
    int tmi, tni;
    tile_coords(P.gm, P.gn, tmi, tni);
    const int m0 = tmi * BM, n0 = tni * BN;
    const int64_t kbase = (int64_t)blockIdx.z * P.K;
    const int64_t klen = min((int64_t)P.K, (int64_t)P.Ktot - kbase);
    const int nk = klen > 0 ? (int)(klen / BK) : 0;   // ragged last split; empty splits write 0
    const float *Ab = TA ? P.A + kbase * P.lda + m0 : P.A + (int64_t)m0 * P.lda + kbase;
    const float *Bb = TB ? P.B + (int64_t)n0 * P.ldb + kbase : P.B + kbase * P.ldb + n0;

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int wave = tid >> 6, lane = tid & 63;
    const int wm = wave >> 1, wn = wave & 1;
    const int kh = lane >> 5, li = lane & 31;

    auto stage = [&](int s) { return smem + s * STAGE; };
    auto compute = [&](const __bf16 *Ah) {
        const __bf16 *Al = Ah + AE, *Bh = Ah + 2 * AE, *Bl = Bh + BE;
#pragma unroll
        for (int ks = 0; ks < BK / 16; ++ks) {
            bf16x8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int o = (wm * WTM + i * 32 + li) * LDK + ks * 16 + kh * 8;
                ah[i] = *reinterpret_cast<const bf16x8 *>(Ah + o);
                if constexpr (SPLIT) al[i] = *reinterpret_cast<const bf16x8 *>(Al + o);
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int o = (wn * WTN + j * 32 + li) * LDK + ks * 16 + kh * 8;
                bh[j] = *reinterpret_cast<const bf16x8 *>(Bh + o);
                if constexpr (SPLIT) bl[j] = *reinterpret_cast<const bf16x8 *>(Bl + o);
            }
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    if constexpr (SPLIT) {
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
                    }
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
                }
        }
    };

    if (nk > 0) {
        // two register stages: every tile's global loads are in flight across TWO compute phases
        // (a single phase of 24 MFMAs does not cover an L2/LLC miss at 2 waves per SIMD)
        float4 ra0[NFA], rb0[NFB], ra1[NFA], rb1[NFB];
        g2r_bf<BM, BK, TA>(Ab, P.lda, 0, tid, ra0);
        g2r_bf<BN, BK, !TB>(Bb, P.ldb, 0, tid, rb0);
        g2r_bf<BM, BK, TA>(Ab, P.lda, min(1, nk - 1), tid, ra1);
        g2r_bf<BN, BK, !TB>(Bb, P.ldb, min(1, nk - 1), tid, rb1);
        r2s_bf<BM, BK, LDK, TA, SPLIT>(stage(0), stage(0) + AE, tid, ra0);
        r2s_bf<BN, BK, LDK, !TB, SPLIT>(stage(0) + 2 * AE, stage(0) + 2 * AE + BE, tid, rb0);
        __syncthreads();
        for (int t = 0; t < nk; t += 2) {
            g2r_bf<BM, BK, TA>(Ab, P.lda, min(t + 2, nk - 1), tid, ra0);
            g2r_bf<BN, BK, !TB>(Bb, P.ldb, min(t + 2, nk - 1), tid, rb0);
            compute(stage(0));
            r2s_bf<BM, BK, LDK, TA, SPLIT>(stage(1), stage(1) + AE, tid, ra1);
            r2s_bf<BN, BK, LDK, !TB, SPLIT>(stage(1) + 2 * AE, stage(1) + 2 * AE + BE, tid, rb1);
            __syncthreads();
            if (t + 1 < nk) {
                g2r_bf<BM, BK, TA>(Ab, P.lda, min(t + 3, nk - 1), tid, ra1);
                g2r_bf<BN, BK, !TB>(Bb, P.ldb, min(t + 3, nk - 1), tid, rb1);
                compute(stage(1));
                r2s_bf<BM, BK, LDK, TA, SPLIT>(stage(0), stage(0) + AE, tid, ra0);
                r2s_bf<BN, BK, LDK, !TB, SPLIT>(stage(0) + 2 * AE, stage(0) + 2 * AE + BE, tid, rb0);
                __syncthreads();
            }
        }
    }

    float *C = P.C + (int64_t)blockIdx.z * P.slab_stride;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = m0 + wm * WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * kh;
                const int col = n0 + wn * WTN + j * 32 + li;
                C[(int64_t)row * P.ldc + col] = epilogue<EPI>(P, row, col, acc[i][j][r]);
            }
}

template <int KIND, int BM, int BN, bool TA, bool TB, int EPI>
void launch_kernel(const GemmP &P, dim3 grid, hipStream_t st) {
    if constexpr (KIND == U2GNN_PREC_F32)
        hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, TA, TB, EPI>), grid, dim3(256), 0, st, P);
    else
        hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, TA, TB, EPI, KIND == U2GNN_PREC_BF16X3>), grid, dim3(256), 0, st,
                           P);
}

template <int KIND, int BM, int BN, bool TA, bool TB>
int launch_epi(const GemmP &P, int epi, int split, hipStream_t st) {
    dim3 grid(P.gm * P.gn, 1, split);
    switch (epi) {
#define U2GNN_CASE(E)                                          \
    case E:                                                    \
        launch_kernel<KIND, BM, BN, TA, TB, E>(P, grid, st);   \
        break;
        U2GNN_CASE(U2GNN_EPI_STORE)
        U2GNN_CASE(U2GNN_EPI_BIAS)
        U2GNN_CASE(U2GNN_EPI_BIAS_DROP_RESID)
        U2GNN_CASE(U2GNN_EPI_BIAS_RELU_DROP)
        U2GNN_CASE(U2GNN_EPI_RELU_DROP_BWD)
        U2GNN_CASE(U2GNN_EPI_ACCUM)
        U2GNN_CASE(U2GNN_EPI_ATTN_DS)
#undef U2GNN_CASE
        default:
            return U2GNN_E_ARG;
    }
    return u2gnn_launch_status();
}

template <int KIND, int BM, int BN>
int launch_layout(const GemmP &P, bool ta, bool tb, int epi, int split, hipStream_t st) {
    if (!ta && tb) return launch_epi<KIND, BM, BN, false, true>(P, epi, split, st);
    if (!ta && !tb) return launch_epi<KIND, BM, BN, false, false>(P, epi, split, st);
    if (ta && !tb) return launch_epi<KIND, BM, BN, true, false>(P, epi, split, st);
    return U2GNN_E_ARG;  // A^T B^T is never needed by the encoder
}

template <int KIND>
int launch_tile(const GemmP &P, int tile, bool ta, bool tb, int epi, int split, hipStream_t st) {
    if (tile == 128) return launch_layout<KIND, 128, 128>(P, ta, tb, epi, split, st);
    return launch_layout<KIND, 64, 64>(P, ta, tb, epi, split, st);
}

inline bool al16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

extern "C" int u2gnn_gemm(const u2gnn_gemm_args *a, void *stream) {
    if (!a || !a->A || !a->B || !a->C) return U2GNN_E_ARG;
    if (a->M <= 0 || a->N <= 0 || a->K <= 0) return U2GNN_E_ARG;
    if (a->epilogue < 0 || a->epilogue > U2GNN_EPI_ATTN_DS) return U2GNN_E_ARG;
    const int prec = a->precision;
    if (prec != U2GNN_PREC_F32 && prec != U2GNN_PREC_BF16X3 && prec != U2GNN_PREC_BF16) return U2GNN_E_ARG;
    const int split = a->split_k < 1 ? 1 : a->split_k;
    if (split > 1 && a->epilogue != U2GNN_EPI_STORE) return U2GNN_E_ARG;
    if (!al16(a->A) || !al16(a->B) || (a->lda & 3) || (a->ldb & 3)) return U2GNN_E_ALIGN;
    const int bk = prec == U2GNN_PREC_F32 ? 16 : 32;
    if (a->K % bk) return U2GNN_E_SHAPE;
    const int e = a->epilogue;
    if ((e == U2GNN_EPI_BIAS || e == U2GNN_EPI_BIAS_DROP_RESID || e == U2GNN_EPI_BIAS_RELU_DROP) && !a->bias)
        return U2GNN_E_ARG;
    if ((e == U2GNN_EPI_BIAS_DROP_RESID || e == U2GNN_EPI_RELU_DROP_BWD || e == U2GNN_EPI_ATTN_DS) && !a->aux0)
        return U2GNN_E_ARG;
    if (e == U2GNN_EPI_ATTN_DS && (!a->aux1 || !a->rowvec)) return U2GNN_E_ARG;
    int tile = a->tile;
    if (tile == 0) {
        const bool can128 = (a->M % 128 == 0) && (a->N % 128 == 0);
        const int64_t blocks128 = can128 ? (a->M / 128) * (a->N / 128) * split : 0;
        tile = (can128 && blocks128 >= 480) ? 128 : 64;
    }
    if (tile != 64 && tile != 128) return U2GNN_E_ARG;
    if (a->M % tile || a->N % tile) return U2GNN_E_SHAPE;
    GemmP P;
    P.A = a->A;
    P.B = a->B;
    P.C = a->C;
    P.lda = a->lda;
    P.ldb = a->ldb;
    P.ldc = a->ldc;
    P.M = (int32_t)a->M;
    P.N = (int32_t)a->N;
    // split z covers k in [z*Kc, min((z+1)*Kc, K)), Kc a multiple of the K tile (the last
    // splits may be short or empty; an empty split writes a zero slab)
    P.K = (int32_t)((a->K + (int64_t)split * bk - 1) / ((int64_t)split * bk) * bk);
    P.Ktot = (int32_t)a->K;
    P.gm = (int32_t)(a->M / tile);
    P.gn = (int32_t)(a->N / tile);
    P.slab_stride = a->slab_stride;
    P.bias = a->bias;
    P.aux0 = a->aux0;
    P.aux1 = a->aux1;
    P.rowvec = a->rowvec;
    P.ld_aux = a->ld_aux;
    P.alpha = a->alpha;
    P.scale_cols = (int32_t)a->scale_cols;
    P.p = a->p_drop;
    P.seed = a->seed;
    hipStream_t st = u2gnn_stream(stream);
    const bool ta = a->trans_a != 0, tb = a->trans_b != 0;
    if (prec == U2GNN_PREC_BF16X3) return launch_tile<U2GNN_PREC_BF16X3>(P, tile, ta, tb, e, split, st);
    if (prec == U2GNN_PREC_BF16) return launch_tile<U2GNN_PREC_BF16>(P, tile, ta, tb, e, split, st);
    return launch_tile<U2GNN_PREC_F32>(P, tile, ta, tb, e, split, st);
}
