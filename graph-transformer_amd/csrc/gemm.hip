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
#include "gemm_common.h"

#include <cmath>
#include <cstring>


namespace {


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

// CLAMP: A elements below +0 are staged as 0 (the signed dropped-probability image read as Pd)
__device__ __forceinline__ float4 clamp0(float4 v) {
    return make_float4(fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f));
}

template <int BM, int BN, int BK, int SA, int SB, bool TA, bool TB, bool CLAMP>
__device__ __forceinline__ void r2s(float *As, float *Bs, int tid, const float4 (&ra_)[BM * BK / 1024],
                                    const float4 (&rb)[BN * BK / 1024]) {
    constexpr int NA = BM * BK / 1024, NB = BN * BK / 1024;
    float4 ra[NA];
#pragma unroll
    for (int i = 0; i < NA; ++i) ra[i] = CLAMP ? clamp0(ra_[i]) : ra_[i];
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
template <int BM, int BN, bool TA, bool TB, int EPI, bool CLAMP>
__global__ void __launch_bounds__(256) gemm_f32_kernel(GemmP P) {
    if constexpr (EPI == U2GNN_EPI_BIAS_DROP_RESID || EPI == U2GNN_EPI_BIAS_RELU_DROP ||
                  EPI == U2GNN_EPI_BIAS_DROP_RESID_LN)
        P.seed = u2gnn_seed(P.seed, P.epoch);   // graph replay: device-resident seed epoch
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
    int zi;
    tile_coords(P.gm, P.gn, tmi, tni, zi);
    const int m0 = tmi * BM, n0 = tni * BN;
    const int64_t kbase = (int64_t)zi * P.K;

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
        r2s<BM, BN, BK, SA, SB, TA, TB, CLAMP>(As0, Bs0, tid, ra, rb);
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
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(b[j], a[i], acc[i][j], 0, 0, 0);  // C^T map
        }
        r2s<BM, BN, BK, SA, SB, TA, TB, CLAMP>(As0 + ((t + 1) & 1) * BK * SA, Bs0 + ((t + 1) & 1) * BK * SB, tid, ra, rb);
        __syncthreads();
    }

    store_tile<EPI>(P, P.C + (int64_t)zi * P.slab_stride, acc, m0 + wm * WTM, n0 + wn * WTN, li, kh,
                    (const PreDS<TN> *)nullptr);
}

// ------------------------------------------------------------------------------------
// split-bf16 MFMA kernel (U2GNN_PREC_BF16X3) and plain bf16 (U2GNN_PREC_BF16)
//
// x = hi + lo with hi = bf16(x), lo = bf16(x - hi) (|x - hi - lo| <= 2^-17 |x|); the product is
// hi*hi + hi*lo + lo*hi on v_mfma_f32_32x32x16_bf16 with fp32 accumulation, i.e. ~2^-16
// relative error per product at 3 bf16 MFMAs (5.3x the fp32-MFMA rate).  fp32 operands are
// split once per block while staging into LDS (register staging; the split is VALU work that
// runs beside the matrix pipe), so HBM/L2 traffic is the fp32 operands themselves.
// LDS images: an operand stored [rows][K] in HBM is staged k-contiguous ([rows][BK+8] bf16: 80-byte
// rows make the ds_read_b128 fragment reads conflict-free); an operand stored [K][rows] is
// staged as it lies, k-major ([BK][rows+32] bf16), and its MFMA fragments are gathered with the
// gfx950 transpose read ds_read_b64_tr_b16 (two per fragment), so neither layout needs a
// register transpose and both keep 16-byte-per-lane coalesced global loads.
// ------------------------------------------------------------------------------------

// LDS bank map of the staging stores (banks = dword mod 32 for ds_write):
//  * [R][K] operands: 8 lanes x 16 B cover one row's 32 k; LDK = 40 bf16 = 20 dwords per row, so
//    the 8 rows of a wave instruction are permuted (0,4,1,5,2,6,3,7): each 16-lane ds_write_b64
//    group then pairs rows 4 apart (16 banks apart), 32 distinct banks;
//  * [K][R] operands: 16 consecutive lanes store 16 x 8 B of one k-row, contiguous.
// Transpose reads: a 32-lane half reads 4 k-rows x 32 columns; a row pitch of R+32 bf16 puts the
// 4 rows 16 dwords apart mod 64, so the 64 dwords of the half hit 64 distinct banks.
template <int BK, int NT>
__device__ __forceinline__ void stage_rk(int tid, int i, int &r, int &kq) {
    const int idx = tid + i * NT;
    const int j = (idx / (BK / 4)) & 7;
    r = (idx / (BK / 4)) - j + ((j >> 1) | ((j & 1) << 2));
    kq = idx % (BK / 4);
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#ifdef U2GNN_EXP_NOSTAGE_A   // experiment: A staged once (upper bound of pre-split A planes)
constexpr bool kStageA = false;
#else
constexpr bool kStageA = true;
#endif
#ifdef U2GNN_EXP_NOSTAGE_B
constexpr bool kStageB = false;
#else
constexpr bool kStageB = true;
#endif

#ifdef U2GNN_EXP_NOSTAGE
#define U2GNN_LOOP_SYNC() ((void)0)
#else
#define U2GNN_LOOP_SYNC() __syncthreads()
#endif

// Global->register staging through raw buffer loads: the per-thread byte offsets (voff) are
// loop-invariant VGPRs, the K-tile advance is one scalar soffset (kt * kstep bytes), so a load
// costs no 64-bit VALU address arithmetic.  The descriptor is built from the block's operand
// base (kernarg + blockIdx only: wave-uniform, no waterfall).
template <int R, int BK, bool T, int NT>
__device__ __forceinline__ void g2r_init(int tid, int64_t ld, int (&voff)[R * BK / (4 * NT)]) {
    constexpr int NF = R * BK / (4 * NT);
    if constexpr (!T) {  // global [R][K]
#pragma unroll
        for (int i = 0; i < NF; ++i) {
            int r, kq;
            stage_rk<BK, NT>(tid, i, r, kq);
            voff[i] = (int)(((int64_t)r * ld + kq * 4) * 4);
        }
    } else {  // global [K][R]: NF k-rows x 4 columns per thread, columns fastest across lanes
        const int mg = tid % (R / 4), kg = tid / (R / 4);
#pragma unroll
        for (int q = 0; q < NF; ++q) voff[q] = (int)(((int64_t)(kg * NF + q) * ld + mg * 4) * 4);
    }
}

template <int NF>
__device__ __forceinline__ void g2r_bf(__amdgpu_buffer_rsrc_t rs, const int (&voff)[NF], int soff,
                                       float4 (&v)[NF]) {
#ifdef U2GNN_EXP_NOLOAD
    if (soff > 0) return;
#endif
#pragma unroll
    for (int i = 0; i < NF; ++i) {
        const u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(rs, voff[i], soff, 0);
        v[i] = make_float4(__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w));
    }
}

// NPL: the planes of each staged element (1: bf16, 2: hi / lo of bf16x3, 3: hi / mid / lo of bf16x6,
// NPL_F16X3: fp16 hi / lo), plane q at p0 + q * pst
constexpr int NPL_F16X3 = 4;
template <int NPL> constexpr int nplanes() { return NPL == NPL_F16X3 ? 2 : NPL; }
template <int NPL>
__device__ __forceinline__ void split_planes(float x0, float x1, float sc, unsigned (&o)[3]) {
    if constexpr (NPL == 3) split3(x0, x1, o[0], o[1], o[2]);
    else if constexpr (NPL == NPL_F16X3) split2h(x0, x1, sc, o[0], o[1]);   // (the pre-scale inside the split)
    else split2<NPL == 2>(x0, x1, o[0], o[1]);
}

template <int R, int BK, int LDK, bool T, int NPL, int NT, bool CLAMP = false>
__device__ __forceinline__ void r2s_bf(__bf16 *p0, int pst, int tid, const float4 (&v_)[R * BK / (4 * NT)],
                                       float sc = 1.f) {
    constexpr int NF = R * BK / (4 * NT);
    float4 v[NF];
#pragma unroll
    for (int i = 0; i < NF; ++i) v[i] = CLAMP ? clamp0(v_[i]) : v_[i];
#ifdef U2GNN_EXP_NOSTAGE
    return;
#endif
#ifdef U2GNN_EXP_NOWRITE   // experiment: loads kept, no split and no LDS write (upper bound of DMA staging)
#pragma unroll
    for (int i = 0; i < NF; ++i) asm volatile("" ::"v"(v[i].x), "v"(v[i].y), "v"(v[i].z), "v"(v[i].w));
    return;
#endif
#pragma unroll
    for (int i = 0; i < NF; ++i) {
        int o;
        if constexpr (!T) {
            int r, kq;
            stage_rk<BK, NT>(tid, i, r, kq);
            o = r * LDK + kq * 4;
        } else {  // k-major image [BK][R + 32]
            const int mg = tid % (R / 4), kg = tid / (R / 4);
            o = (kg * NF + i) * (R + 32) + mg * 4;
        }
        unsigned a[3], b[3];
        split_planes<NPL>(v[i].x, v[i].y, sc, a);
        split_planes<NPL>(v[i].z, v[i].w, sc, b);
#pragma unroll
        for (int q = 0; q < nplanes<NPL>(); ++q) *reinterpret_cast<uint2 *>(p0 + q * pst + o) = make_uint2(a[q], b[q]);
    }
}

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// One 32x32x16 MFMA operand fragment (lane l: row r0 + l%32, k = ks*16 + 8*(l/32) .. +7).
template <int R, int LDK, bool T>
__device__ __forceinline__ bf16x8 ld_frag(const __bf16 *img, int r0, int ks, int lane) {
    if constexpr (!T) {
        return *reinterpret_cast<const bf16x8 *>(img + (r0 + (lane & 31)) * LDK + ks * 16 + (lane >> 5) * 8);
    } else {
        // ds_read_b64_tr_b16: within each 16-lane group, lane 4q+p addresses k-row q, columns
        // 4p..4p+3 of a 4 x 16 block and receives column (lane % 16) of the 4 rows
        constexpr int S = R + 32;
        const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
        const __bf16 *a = img + (ks * 16 + (g >> 1) * 8 + q) * S + r0 + (g & 1) * 16 + 4 * p;
        const s16x4 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)a);
        const s16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(a + 4 * S));
        const s16x4 v[2] = {x0, x1};
        return __builtin_bit_cast(bf16x8, v);
    }
}

// The main loop and epilogue of one output tile (tile coordinates from the caller: the plain launch's
// XCD-aware map, or the grouped launch's job walk).
// 16-bit planes held per staged operand: two for bf16 / bf16x3 (the bf16 kind leaves its second plane unused, so
// both kinds share one LDS layout) and f16x3, three for bf16x6
template <int NPL> constexpr int planes_of() { return NPL < 2 ? 2 : nplanes<NPL>(); }
// bf16 elements of the kernel's LDS image (two stages of the planes of both operands)
template <int BM, int BN, int BK, bool TA, bool TB, int NPL = 2>
constexpr int bf16_smem_elems() {
    constexpr int LDK = BK + 8;
    constexpr int AE = TA ? BK * (BM + 32) : BM * LDK;
    constexpr int BE = !TB ? BK * (BN + 32) : BN * LDK;
    return 2 * planes_of<NPL>() * (AE + BE);
}

// dS epilogue through LDS (the C4 dS product: 128 x 128 blocks of 2 x 2 waves, 32-deep K step): each wave's
// 64 x 64 result goes to LDS in the MFMA layout and comes back row-contiguous (16 lanes x 16 B per row, 4 rows
// per instruction), so the probability-image loads and the dS stores cover whole 128-byte lines per
// instruction instead of 32 rows x 32 B; the per-element arithmetic is epilogue4's (same bits).  The live dS
// probe in the C4 step: 85 vs 93-94 us, step 2.922-2.926 vs 2.934-2.976 ms (profiles/r05/ab_ds_lds_epilogue.txt).
// The first half's operands are fetched before the main loop (as the MFMA-layout form did for slice 0).
constexpr int DSL_PITCH = 68;   // floats per LDS row (64 + 4)
struct DsPre {
    float4 p[8];
    float dl[8];
};
__device__ __forceinline__ void ds_lds_fetch(const GemmP &P, int r0, int c0, int lane, int it0, DsPre &f) {
    const int rl = lane >> 4, cl = (lane & 15) * 4;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int row = r0 + rl + 4 * (it0 + q);
        f.p[q] = ld4(P.aux0 + (int64_t)row * P.ld_aux + c0 + cl);
        f.dl[q] = P.rowvec[row];
    }
}
__device__ __forceinline__ void ds_lds_store(const GemmP &P, float *C, const f32x16 (&acc)[2][2], int r0, int c0,
                                             int wave, int lane, __bf16 *smem, const DsPre &pre) {
    constexpr int E = U2GNN_EPI_ATTN_DS_SIGNED;
    const int li = lane & 31, kh = lane >> 5;
    DsPre hi;
    ds_lds_fetch(P, r0, c0, lane, 8, hi);   // the second half's operands in flight under the first half
    float *L = reinterpret_cast<float *>(smem) + wave * 64 * DSL_PITCH;
    __syncthreads();   // every wave is done with the main loop's LDS images
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int g = 0; g < 4; ++g)
                *reinterpret_cast<float4 *>(L + (32 * i + li) * DSL_PITCH + 32 * j + 8 * g + 4 * kh) =
                    make_float4(acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]);
    __syncthreads();
    const int rl = lane >> 4, cl = (lane & 15) * 4;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int r = rl + 4 * q;
        const float4 v = *reinterpret_cast<const float4 *>(L + r * DSL_PITCH + cl);
        *reinterpret_cast<float4 *>(C + (int64_t)(r0 + r) * P.ldc + c0 + cl) =
            epilogue4<E>(P, r0 + r, c0 + cl, v, pre.p[q], z4, 0u, pre.dl[q]);
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int r = rl + 4 * (q + 8);
        const float4 v = *reinterpret_cast<const float4 *>(L + r * DSL_PITCH + cl);
        *reinterpret_cast<float4 *>(C + (int64_t)(r0 + r) * P.ldc + c0 + cl) =
            epilogue4<E>(P, r0 + r, c0 + cl, v, hi.p[q], z4, 0u, hi.dl[q]);
    }
}

template <int BM, int BN, int WM, int WN, int BK, bool TA, bool TB, int EPI, int NPL, bool CLAMP>
__device__ __forceinline__ void gemm_bf16_body(const GemmP &P, int tmi, int tni, int zi, __bf16 *smem) {
    constexpr int NT = 64 * WM * WN;
    constexpr int LDK = BK + 8;
    constexpr int WTM = BM / WM, WTN = BN / WN;
    constexpr int TM = WTM / 32, TN = WTN / 32;
    constexpr int NFA = BM * BK / (4 * NT), NFB = BN * BK / (4 * NT);
    constexpr int AE = TA ? BK * (BM + 32) : BM * LDK;    // elements per plane, per operand
    constexpr int BE = !TB ? BK * (BN + 32) : BN * LDK;
    constexpr int PL = planes_of<NPL>();
    constexpr int STAGE = PL * (AE + BE);  // the planes of A, then those of B

    const int tid = threadIdx.x;
    const int m0 = tmi * BM, n0 = tni * BN;
    const int64_t kbase = (int64_t)zi * P.K;
    const int64_t klen = min((int64_t)P.K, (int64_t)P.Ktot - kbase);
    const int nk = klen > 0 ? (int)(klen / BK) : 0;   // ragged last split; empty splits write 0
    const float *Ab = TA ? P.A + kbase * P.lda + m0 : P.A + (int64_t)m0 * P.lda + kbase;
    const float *Bb = TB ? P.B + (int64_t)n0 * P.ldb + kbase : P.B + kbase * P.ldb + n0;
    const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void *)Ab, 0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc((void *)Bb, 0, 0x7fffffff, 0x00020000);
    const int kstepA = TA ? (int)(BK * P.lda * 4) : BK * 4;   // bytes per K tile
    const int kstepB = TB ? BK * 4 : (int)(BK * P.ldb * 4);
    int voA[NFA], voB[NFB];
    g2r_init<BM, BK, TA, NT>(tid, P.lda, voA);
    g2r_init<BN, BK, !TB, NT>(tid, P.ldb, voB);

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int wave = tid >> 6, lane = tid & 63;
    const int wm = wave / WN, wn = wave % WN;
    const int kh = lane >> 5, li = lane & 31;

    auto stage = [&](int s) { return smem + s * STAGE; };
    auto compute = [&](const __bf16 *Ah) {
        const __bf16 *Bh = Ah + PL * AE;
#pragma unroll
        for (int ks = 0; ks < BK / 16; ++ks) {
            constexpr int NP = nplanes<NPL>();
            bf16x8 a[NP][TM], b[NP][TN];
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int q = 0; q < NP; ++q) a[q][i] = ld_frag<BM, LDK, TA>(Ah + q * AE, wm * WTM + i * 32, ks, lane);
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int q = 0; q < NP; ++q) b[q][j] = ld_frag<BN, LDK, !TB>(Bh + q * BE, wn * WTN + j * 32, ks, lane);
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    // B fragment first: the accumulator holds the tile transposed, so each lane
                    // owns 4 consecutive output columns of one row (16-byte epilogue accesses).
                    // Smallest terms first: bf16x6 mid.mid, hi.lo, lo.hi, hi.mid, mid.hi; bf16x3 hi.lo, lo.hi;
                    // then hi.hi (f16x3: hi.lo, lo.hi, hi.hi on the fp16 matrix cores, same fragment layout)
                    if constexpr (NPL == NPL_F16X3) {
                        const auto h = [](bf16x8 v) { return __builtin_bit_cast(f16x8, v); };
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(h(b[0][j]), h(a[1][i]), acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(h(b[1][j]), h(a[0][i]), acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(h(b[0][j]), h(a[0][i]), acc[i][j], 0, 0, 0);
                    } else {
                        if constexpr (NPL == 3) {
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[1][j], a[1][i], acc[i][j], 0, 0, 0);
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[0][j], a[2][i], acc[i][j], 0, 0, 0);
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[2][j], a[0][i], acc[i][j], 0, 0, 0);
                        }
                        if constexpr (NPL >= 2) {
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[0][j], a[1][i], acc[i][j], 0, 0, 0);
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[1][j], a[0][i], acc[i][j], 0, 0, 0);
                        }
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[0][j], a[0][i], acc[i][j], 0, 0, 0);
                    }
                }
        }
    };

    constexpr bool DSL = EPI == U2GNN_EPI_ATTN_DS_SIGNED && BM == 128 && BN == 128 && WM == 2 && WN == 2 && BK == 32;
    static_assert(!DSL || 4 * 64 * DSL_PITCH * 4 <= 2 * bf16_smem_elems<BM, BN, BK, TA, TB, NPL>(), "dS LDS epilogue image");
    DsPre dsl;
    if constexpr (DSL) ds_lds_fetch(P, m0 + wm * WTM, n0 + wn * WTN, lane, 0, dsl);
    PreDS<TN> pre;
    const bool use_pre = !DSL && ((EPI == U2GNN_EPI_ATTN_DS && P.keep != nullptr) || ds_signed<EPI>);
    if (use_pre) prefetch_ds<EPI>(P, m0 + wm * WTM + li, n0 + wn * WTN, kh, pre);
    // 64 x 64 tiles with row-operand epilogues: the slice's residual / bias / accumulator / ReLU operands
    // requested before the main loop (the short K loops of these products do not hide the epilogue's round
    // trip): C4 3.010-3.027 vs 3.027-3.051 ms, C5 0.804 vs 0.808-0.809 ms per step (one session each)
    constexpr bool PRE_AUX = TM == 1 && TN == 1 &&
                             (EPI == U2GNN_EPI_BIAS_DROP_RESID || EPI == U2GNN_EPI_BIAS_DROP_RESID_LN ||
                              EPI == U2GNN_EPI_RELU_DROP_BWD || EPI == U2GNN_EPI_ACCUM);   // bias-only epilogues
                                                                                           // too: neutral
    EpiSlice<pre_aux_fetch<EPI>, TN> pa;
    if constexpr (PRE_AUX) fetch_slice<pre_aux_fetch<EPI>>(P, m0 + wm * WTM + li, n0 + wn * WTN, kh, pa);
    if (nk > 0) {
        // two register stages: every tile's global loads are in flight across TWO compute phases
        // (a single phase of 24 MFMAs does not cover an L2/LLC miss at 2 waves per SIMD)
        float4 ra0[NFA], rb0[NFB], ra1[NFA], rb1[NFB];
        g2r_bf<NFA>(rsA, voA, (0) * kstepA, ra0);
        g2r_bf<NFB>(rsB, voB, (0) * kstepB, rb0);
        g2r_bf<NFA>(rsA, voA, (min(1, nk - 1)) * kstepA, ra1);
        g2r_bf<NFB>(rsB, voB, (min(1, nk - 1)) * kstepB, rb1);
        r2s_bf<BM, BK, LDK, TA, NPL, NT, CLAMP>(stage(0), AE, tid, ra0, P.h3_sa);
        r2s_bf<BN, BK, LDK, !TB, NPL, NT>(stage(0) + PL * AE, BE, tid, rb0, P.h3_sb);
        __syncthreads();
        for (int t = 0; t < nk; t += 2) {
            if constexpr (kStageA) g2r_bf<NFA>(rsA, voA, (min(t + 2, nk - 1)) * kstepA, ra0);
            if constexpr (kStageB) g2r_bf<NFB>(rsB, voB, (min(t + 2, nk - 1)) * kstepB, rb0);
            compute(stage(0));
            if constexpr (kStageA) r2s_bf<BM, BK, LDK, TA, NPL, NT, CLAMP>(stage(1), AE, tid, ra1, P.h3_sa);
            if constexpr (kStageB) r2s_bf<BN, BK, LDK, !TB, NPL, NT>(stage(1) + PL * AE, BE, tid, rb1, P.h3_sb);
            U2GNN_LOOP_SYNC();
            if (t + 1 < nk) {
                if constexpr (kStageA) g2r_bf<NFA>(rsA, voA, (min(t + 3, nk - 1)) * kstepA, ra1);
                if constexpr (kStageB) g2r_bf<NFB>(rsB, voB, (min(t + 3, nk - 1)) * kstepB, rb1);
                compute(stage(1));
                if constexpr (kStageA) r2s_bf<BM, BK, LDK, TA, NPL, NT, CLAMP>(stage(0), AE, tid, ra0, P.h3_sa);
                if constexpr (kStageB) r2s_bf<BN, BK, LDK, !TB, NPL, NT>(stage(0) + PL * AE, BE, tid, rb0, P.h3_sb);
                U2GNN_LOOP_SYNC();
            }
        }
    }

    if constexpr (NPL == NPL_F16X3) {   // undo the operand pre-scales (exact)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[i][j] *= P.h3_inv;
    }
    if constexpr (DSL) {
        ds_lds_store(P, P.C + (int64_t)zi * P.slab_stride, acc, m0 + wm * WTM, n0 + wn * WTN, wave, lane, smem, dsl);
        return;
    }
    store_tile<EPI>(P, P.C + (int64_t)zi * P.slab_stride, acc, m0 + wm * WTM, n0 + wn * WTN, li, kh,
                    use_pre ? &pre : nullptr, PRE_AUX ? &pa : nullptr);
}

template <int BM, int BN, int WM, int WN, int BK, bool TA, bool TB, int EPI, bool SPLIT, bool CLAMP>
__global__ void __launch_bounds__(64 * WM * WN) gemm_bf16_kernel(GemmP P) {
    if constexpr (EPI == U2GNN_EPI_BIAS_DROP_RESID || EPI == U2GNN_EPI_BIAS_RELU_DROP ||
                  EPI == U2GNN_EPI_BIAS_DROP_RESID_LN)
        P.seed = u2gnn_seed(P.seed, P.epoch);   // graph replay: device-resident seed epoch
    __shared__ __attribute__((aligned(16))) __bf16 smem[bf16_smem_elems<BM, BN, BK, TA, TB>()];
    int tmi, tni, zi;
    tile_coords(P.gm, P.gn, tmi, tni, zi);
    gemm_bf16_body<BM, BN, WM, WN, BK, TA, TB, EPI, SPLIT ? 2 : 1, CLAMP>(P, tmi, tni, zi, smem);
}

// U2GNN_PREC_BF16X6: the same body over three planes per operand (16-deep K step, so that the 256x128
// tile's two stages of six planes fit: 108 KB)
template <int BM, int BN, int WM, int WN, bool TA, bool TB, int EPI, bool CLAMP>
__global__ void __launch_bounds__(64 * WM * WN) gemm_bf16x6_kernel(GemmP P) {
    if constexpr (EPI == U2GNN_EPI_BIAS_DROP_RESID || EPI == U2GNN_EPI_BIAS_RELU_DROP ||
                  EPI == U2GNN_EPI_BIAS_DROP_RESID_LN)
        P.seed = u2gnn_seed(P.seed, P.epoch);   // graph replay: device-resident seed epoch
    __shared__ __attribute__((aligned(16))) __bf16 smem[bf16_smem_elems<BM, BN, 16, TA, TB, 3>()];
    int tmi, tni, zi;
    tile_coords(P.gm, P.gn, tmi, tni, zi);
    gemm_bf16_body<BM, BN, WM, WN, 16, TA, TB, EPI, 3, CLAMP>(P, tmi, tni, zi, smem);
}

// U2GNN_PREC_F16X3: the bf16x3 body over two fp16 planes per operand (fp16 MFMA), the forward products only
template <int BM, int BN, int WM, int WN, int BK, bool TA, bool TB, int EPI, bool CLAMP>
__global__ void __launch_bounds__(64 * WM * WN) gemm_f16x3_kernel(GemmP P) {
    if constexpr (EPI == U2GNN_EPI_BIAS_DROP_RESID || EPI == U2GNN_EPI_BIAS_RELU_DROP ||
                  EPI == U2GNN_EPI_BIAS_DROP_RESID_LN)
        P.seed = u2gnn_seed(P.seed, P.epoch);   // graph replay: device-resident seed epoch
    __shared__ __attribute__((aligned(16))) __bf16 smem[bf16_smem_elems<BM, BN, BK, TA, TB, NPL_F16X3>()];
    int tmi, tni, zi;
    tile_coords(P.gm, P.gn, tmi, tni, zi);
    gemm_bf16_body<BM, BN, WM, WN, BK, TA, TB, EPI, NPL_F16X3, CLAMP>(P, tmi, tni, zi, smem);
}

// Grouped launch (u2gnn_gemm_group): several STORE products of one tile shape, each A^T B (the weight
// gradients, dK), A^T B over the clamped signed image (dV) or A B (dQ).  The XCD-aware logical id runs
// over the whole grid; job j owns ids [start[j], start[j+1]) and maps its local id to a tile exactly as
// its own launch would, with the body of its own layout (same tile arithmetic, hence the same bits).  The
// three bodies share one LDS image sized for the largest.
constexpr int GG_MAX = 8;
enum GgLayout : int32_t { GG_TA = 0, GG_TA_CLAMP = 1, GG_NN = 2 };
struct GemmGroup {
    GemmP p[GG_MAX];
    int32_t start[GG_MAX + 1];
    int32_t layout[GG_MAX];
    int32_t n;
};

template <int BM, int BN, int WM, int WN, int BK, bool SPLIT>
__global__ void __launch_bounds__(64 * WM * WN) gemm_bf16_group_kernel(GemmGroup G) {
    constexpr int E_TA = bf16_smem_elems<BM, BN, BK, true, false>(), E_NN = bf16_smem_elems<BM, BN, BK, false, false>();
    __shared__ __attribute__((aligned(16))) __bf16 smem[E_TA > E_NN ? E_TA : E_NN];
    const int w = xcd_wgid();
    int j = 0;
    while (j + 1 < G.n && w >= G.start[j + 1]) ++j;
    const GemmP &P = G.p[j];
    int tmi, tni, zi;
    tile_of(P.gm, P.gn, w - G.start[j], tmi, tni, zi);
    const int lay = G.layout[j];
    if (lay == GG_NN)
        gemm_bf16_body<BM, BN, WM, WN, BK, false, false, U2GNN_EPI_STORE, SPLIT ? 2 : 1, false>(P, tmi, tni, zi, smem);
    else if (lay == GG_TA_CLAMP)
        gemm_bf16_body<BM, BN, WM, WN, BK, true, false, U2GNN_EPI_STORE, SPLIT ? 2 : 1, true>(P, tmi, tni, zi, smem);
    else
        gemm_bf16_body<BM, BN, WM, WN, BK, true, false, U2GNN_EPI_STORE, SPLIT ? 2 : 1, false>(P, tmi, tni, zi, smem);
}

// bf16 K-step variants: 0 = BK 32 (2 blocks/CU at 128x128), 1 = BK 16 (40 KB LDS, 140-152
// VGPRs: 3 blocks/CU; the skinny weight-gradient products run faster at that occupancy).
// Measured and not kept (tools/gemm_bench.py, round 1): BK 64 at one block per CU (-30..-45 %),
// staging written after the barrier from one register set (+-2 %).
template <int VAR> constexpr int CFG_BK = VAR == 1 ? 16 : 32;

template <int KIND, int BM, int BN, int VAR, bool TA, bool TB, int EPI, bool CLAMP = false>
void launch_kernel(const GemmP &P, dim3 grid, hipStream_t st) {
    if constexpr (KIND == U2GNN_PREC_F32) {
        hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, TA, TB, EPI, CLAMP>), grid, dim3(256), 0, st, P);
    } else if constexpr (KIND == U2GNN_PREC_BF16X6) {
        constexpr int WM = BM == 256 ? 4 : 2, WN = 2;
        hipLaunchKernelGGL((gemm_bf16x6_kernel<BM, BN, WM, WN, TA, TB, EPI, CLAMP>), grid, dim3(64 * WM * WN), 0, st, P);
    } else if constexpr (KIND == U2GNN_PREC_F16X3) {
        constexpr int WM = BM == 256 ? 4 : 2, WN = 2;
        hipLaunchKernelGGL((gemm_f16x3_kernel<BM, BN, WM, WN, CFG_BK<VAR>, TA, TB, EPI, CLAMP>), grid,
                           dim3(64 * WM * WN), 0, st, P);
    } else {
        constexpr int WM = BM == 256 ? 4 : 2, WN = 2;   // 256x128 tiles run 8 waves (4x2)
        hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, WM, WN, CFG_BK<VAR>, TA, TB, EPI,
                                             KIND == U2GNN_PREC_BF16X3, CLAMP>),
                           grid, dim3(64 * WM * WN), 0, st, P);
    }
}

// the kinds built for the forward products only (A never transposed, x6_epi's epilogues)
constexpr bool fwd_kind(int k) { return k == U2GNN_PREC_BF16X6 || k == U2GNN_PREC_F16X3; }
// the epilogues the bf16x6 / f16x3 kernels are built for (the forward products; u2gnn_gemm refuses the others)
constexpr bool x6_epi(int e) {
    return e == U2GNN_EPI_STORE || e == U2GNN_EPI_BIAS || e == U2GNN_EPI_BIAS_DROP_RESID ||
           e == U2GNN_EPI_BIAS_RELU_DROP || e == U2GNN_EPI_ACCUM || e == U2GNN_EPI_STORE_ROWSTAT ||
           e == U2GNN_EPI_BIAS_DROP_RESID_LN;
}

template <int KIND, int BM, int BN, int VAR, bool TA, bool TB>
int launch_epi(const GemmP &P, int epi, int split, bool clamp_a, hipStream_t st) {
    dim3 grid(P.gm * P.gn * split);
    if (clamp_a) {   // the P.V / dV products over the signed probability image: STORE, B not transposed
        if constexpr (TB) {
            return U2GNN_E_ARG;
        } else {
            if (epi != U2GNN_EPI_STORE) return U2GNN_E_ARG;
            launch_kernel<KIND, BM, BN, VAR, TA, TB, U2GNN_EPI_STORE, true>(P, grid, st);
            return u2gnn_launch_status();
        }
    }
    if (fwd_kind(KIND) && !x6_epi(epi)) return U2GNN_E_ARG;
    switch (epi) {
#define U2GNN_CASE(E)                                                                    \
    case E:                                                                              \
        if constexpr (!fwd_kind(KIND) || x6_epi(E)) launch_kernel<KIND, BM, BN, VAR, TA, TB, E>(P, grid, st); \
        break;
        U2GNN_CASE(U2GNN_EPI_STORE)
        U2GNN_CASE(U2GNN_EPI_BIAS)
        U2GNN_CASE(U2GNN_EPI_BIAS_DROP_RESID)
        U2GNN_CASE(U2GNN_EPI_BIAS_RELU_DROP)
        U2GNN_CASE(U2GNN_EPI_RELU_DROP_BWD)
        U2GNN_CASE(U2GNN_EPI_ACCUM)
        U2GNN_CASE(U2GNN_EPI_ATTN_DS)
        U2GNN_CASE(U2GNN_EPI_STORE_ROWDOT)
#undef U2GNN_CASE
        case U2GNN_EPI_STORE_ROWSTAT:   // the attention scores and their row partials, bf16 kinds only
            if constexpr (KIND != U2GNN_PREC_F32 && !TA && TB)
                launch_kernel<KIND, BM, BN, VAR, TA, TB, U2GNN_EPI_STORE_ROWSTAT>(P, grid, st);
            else
                return U2GNN_E_ARG;
            break;
        case U2GNN_EPI_ATTN_DS_SIGNED:   // delta as STORE_ROWDOT partials: its own instantiation
            if constexpr (fwd_kind(KIND)) return U2GNN_E_ARG;
            else if (P.rowvec_parts > 1)
                launch_kernel<KIND, BM, BN, VAR, TA, TB, EPI_DS_SIGNED_PARTS>(P, grid, st);
            else
                launch_kernel<KIND, BM, BN, VAR, TA, TB, U2GNN_EPI_ATTN_DS_SIGNED>(P, grid, st);
            break;
        case U2GNN_EPI_BIAS_DROP_RESID_LN:   // row-complete 64 x 64 blocks, NT, bf16 kinds only
            if constexpr (KIND != U2GNN_PREC_F32 && BM == 64 && BN == 64 && !TA && TB)
                launch_kernel<KIND, BM, BN, VAR, TA, TB, U2GNN_EPI_BIAS_DROP_RESID_LN>(P, grid, st);
            else
                return U2GNN_E_ARG;
            break;
        default:
            return U2GNN_E_ARG;
    }
    return u2gnn_launch_status();
}

template <int KIND, int BM, int BN, int VAR = 0>
int launch_layout(const GemmP &P, bool ta, bool tb, int epi, int split, bool clamp_a, hipStream_t st) {
    if (!ta && tb) return launch_epi<KIND, BM, BN, VAR, false, true>(P, epi, split, clamp_a, st);
    if (!ta && !tb) return launch_epi<KIND, BM, BN, VAR, false, false>(P, epi, split, clamp_a, st);
    if constexpr (!fwd_kind(KIND))   // (bf16x6 / f16x3: the forward products, A never transposed)
        if (ta && !tb) return launch_epi<KIND, BM, BN, VAR, true, false>(P, epi, split, clamp_a, st);
    return U2GNN_E_ARG;  // A^T B^T is never needed by the encoder
}

template <int KIND>
int launch_tile(const GemmP &P, int tile, bool ta, bool tb, int epi, int split, bool clamp_a, hipStream_t st) {
    if constexpr (KIND != U2GNN_PREC_F32) {
        if (tile == 256) return launch_layout<KIND, 256, 128>(P, ta, tb, epi, split, clamp_a, st);
        if (tile == 129) return launch_layout<KIND, 128, 128, 1>(P, ta, tb, epi, split, clamp_a, st);
    }
    if (tile == 128) return launch_layout<KIND, 128, 128>(P, ta, tb, epi, split, clamp_a, st);
    return launch_layout<KIND, 64, 64>(P, ta, tb, epi, split, clamp_a, st);
}

inline bool al16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

namespace {

// validated launch description of one u2gnn_gemm call
struct GemmPlan {
    GemmP P;
    int tile, split, prec, epi;
    bool ta, tb, clamp;
};

int gemm_plan(const u2gnn_gemm_args *a, GemmPlan &G) {
    if (!a) return U2GNN_E_ARG;
    // pre-split (x2) operands were the round-1/2 GEMM experiments (gemm_x2.hip / gemm_x3.hip, DESIGN.md 5.1,
    // 5.3), measured slower than this kernel and removed in round 4 together with the recomputed-P dS epilogue
    // that served them (ABI v13); the x2 OUTPUT (Cx2) stays on the path
    if (a->a_x2 || a->b_x2 || a->epilogue == U2GNN_EPI_ATTN_DS_RECOMP) return U2GNN_E_ARG;
    if (!a->A || !a->B) return U2GNN_E_ARG;
    if (!a->C && !a->Cx2) return U2GNN_E_ARG;
    if (a->M <= 0 || a->N <= 0 || a->K <= 0) return U2GNN_E_ARG;
    if (a->epilogue < 0 || a->epilogue > U2GNN_EPI_STORE_ROWSTAT) return U2GNN_E_ARG;
    const int prec = a->precision;
    if (prec != U2GNN_PREC_F32 && prec != U2GNN_PREC_BF16X3 && prec != U2GNN_PREC_BF16 && prec != U2GNN_PREC_BF16X6 &&
        prec != U2GNN_PREC_F16X3)
        return U2GNN_E_ARG;
    if (fwd_kind(prec) && (a->trans_a || !x6_epi(a->epilogue))) return U2GNN_E_ARG;
    if (prec == U2GNN_PREC_F16X3 ? (a->h3_exp_a < -24 || a->h3_exp_a > 24 || a->h3_exp_b < -24 || a->h3_exp_b > 24)
                                 : (a->h3_exp_a != 0 || a->h3_exp_b != 0))
        return U2GNN_E_ARG;
    const int split = a->split_k < 1 ? 1 : a->split_k;
    if (split > 1 && (a->epilogue != U2GNN_EPI_STORE || a->Cx2 || !a->C)) return U2GNN_E_ARG;
    if (!al16(a->A) || !al16(a->B) || (a->lda & 3) || (a->ldb & 3)) return U2GNN_E_ALIGN;
    const int bk = (prec == U2GNN_PREC_F32 || prec == U2GNN_PREC_BF16X6 || a->tile == 129) ? 16 : 32;   // K step
    if (a->K % bk) return U2GNN_E_SHAPE;
    if (prec != U2GNN_PREC_F32) {   // bf16 staging addresses operands by 32-bit buffer offsets
        const int64_t span = ((int64_t)a->K + 256) * (a->lda > a->ldb ? a->lda : a->ldb) * 4;
        if (span >= (int64_t)INT32_MAX) return U2GNN_E_SHAPE;
    }
    // 16-byte epilogue: C, bias and aux rows are read/written as float4; x2 output as 8-byte pairs
    if ((a->C && (!al16(a->C) || (a->ldc & 3))) || (split > 1 && (a->slab_stride & 3))) return U2GNN_E_ALIGN;
    if (a->Cx2 && (!al16(a->Cx2) || (a->ldcx2 & 15) || (a->N & 7))) return U2GNN_E_ALIGN;
    if (a->cx2_col0 < 0 || (a->cx2_col0 & 7)) return U2GNN_E_ARG;
    if ((a->bias && !al16(a->bias)) || (a->aux0 && !al16(a->aux0)) || (a->aux1 && !al16(a->aux1)) ||
        ((a->aux0 || a->aux1) && (a->ld_aux & 3)))
        return U2GNN_E_ALIGN;
    const int e = a->epilogue;
    if ((e == U2GNN_EPI_BIAS || e == U2GNN_EPI_BIAS_DROP_RESID || e == U2GNN_EPI_BIAS_RELU_DROP ||
         e == U2GNN_EPI_BIAS_DROP_RESID_LN) && !a->bias)
        return U2GNN_E_ARG;
    if (e == U2GNN_EPI_BIAS_DROP_RESID_LN) {   // row-complete 64-column tiles only (the d <= 64 encoders)
        if (prec == U2GNN_PREC_F32 || split != 1 || a->N != 64 || (a->tile != 0 && a->tile != 64) ||
            a->trans_a || !a->trans_b || !a->aux0 || !a->ln_gamma || !a->ln_beta || !a->ln_y || !a->ln_mean ||
            !a->ln_rstd || a->ln_d < 1 || a->ln_d > 64 || a->ln_rows < 0)
            return U2GNN_E_ARG;
        if (!al16(a->ln_y) || (a->ln_ldy & 3)) return U2GNN_E_ALIGN;
    }
    if ((e == U2GNN_EPI_BIAS_DROP_RESID || e == U2GNN_EPI_BIAS_DROP_RESID_LN || e == U2GNN_EPI_RELU_DROP_BWD ||
         e == U2GNN_EPI_STORE_ROWDOT || e == U2GNN_EPI_ATTN_DS ||
         e == U2GNN_EPI_ATTN_DS_SIGNED) && !a->aux0)
        return U2GNN_E_ARG;
    // (C required and no x2 copy: the 128 x 128 dS kernel stages its result through LDS into C alone)
    if (e == U2GNN_EPI_ATTN_DS_SIGNED && (!a->rowvec || !(a->p_drop < 1.f) || !a->C || a->Cx2)) return U2GNN_E_ARG;
    if (a->rowvec_parts > 1 && (e != U2GNN_EPI_ATTN_DS_SIGNED || a->ld_rowvec < a->M)) return U2GNN_E_ARG;
    if (e == U2GNN_EPI_STORE_ROWDOT &&
        (split != 1 || a->Cx2 || !a->aux0 || !a->rowpart || a->ld_rowpart < a->M || (a->N & 63)))
        return U2GNN_E_ARG;
    if (e == U2GNN_EPI_STORE_ROWSTAT) {
        if (prec == U2GNN_PREC_F32 || split != 1 || a->Cx2 || !a->C || !a->rowpart || a->trans_a ||
            !a->trans_b || a->n_valid < 1 || a->n_valid > a->N || a->ld_rowpart < a->N / 32)
            return U2GNN_E_ARG;
        if ((uintptr_t)a->rowpart & 7) return U2GNN_E_ALIGN;
    }
    if (a->clamp_a && (e != U2GNN_EPI_STORE || a->trans_b)) return U2GNN_E_ARG;
    if (e == U2GNN_EPI_ATTN_DS && ((!a->aux1 && !a->keep) || !a->rowvec)) return U2GNN_E_ARG;
    if (e == U2GNN_EPI_ATTN_DS && a->keep && (a->ld_keep * 32 < a->N || !(a->p_drop < 1.f))) return U2GNN_E_ARG;
    int tile = a->tile;
    if (tile == 0) {
        const bool can128 = (a->M % 128 == 0) && (a->N % 128 == 0);
        const int64_t blocks128 = can128 ? (a->M / 128) * (a->N / 128) * split : 0;
        tile = (can128 && blocks128 >= 480) ? 128 : 64;
        // token-sized products (neighbour attention: M = N(k+1) rows) have 3+ waves of 256x128
        // blocks: the 8-wave tile's higher intensity wins there for plain store / accumulate
        // epilogues (measured: dH.W1 403 -> 322 us), not for the fused bias/dropout/ReLU ones
        // (ReLU-backward 464 -> 529 us).  Node-sized products (C4: at most 722 such blocks) keep
        // the 128 tile, measured faster for them.
        if (prec != U2GNN_PREC_F32 && (e == U2GNN_EPI_STORE || e == U2GNN_EPI_ACCUM) && a->M % 256 == 0 &&
            a->N % 128 == 0 &&
            (a->M / 256) * (a->N / 128) * split >= U2GNN_BIG_TILE_BLOCKS)
            tile = 256;
    }
    // tile codes: 64, 128 (square), 256 (256x128, 8 waves), 129 (128x128 with a 16-deep K step)
    if (tile != 64 && tile != 128 && tile != 256 && tile != 129) return U2GNN_E_ARG;
    if ((tile == 256 || tile == 129) && prec == U2GNN_PREC_F32) return U2GNN_E_ARG;
    const int tm_ = tile == 129 ? 128 : tile;
    const int tile_n = tm_ == 256 ? 128 : tm_;
    if (a->M % tm_ || a->N % tile_n) return U2GNN_E_SHAPE;
    GemmP P;
    std::memset(&P, 0, sizeof(P));
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
    const int kq = bk;   // K granule of one split
    P.K = (int32_t)((a->K + (int64_t)split * kq - 1) / ((int64_t)split * kq) * kq);
    P.Ktot = (int32_t)a->K;
    P.gm = (int32_t)(a->M / tm_);
    P.gn = (int32_t)(a->N / tile_n);
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
    P.epoch = u2gnn_cur_epoch();
    P.keep = e == U2GNN_EPI_ATTN_DS ? a->keep : nullptr;
    P.ld_keep = a->ld_keep;
    P.Cx2 = static_cast<__bf16 *>(a->Cx2);
    P.ldcx2 = a->ldcx2;
    P.cx2_col0 = a->cx2_col0;
    P.cx2_h3 = prec == U2GNN_PREC_F16X3 ? std::ldexp(1.f, U2GNN_H3_X2_EXP) : 0.f;
    P.n_valid = (int32_t)a->n_valid;
    P.rowpart = a->rowpart;
    P.ld_rowpart = a->ld_rowpart;
    P.rowvec_parts = a->rowvec_parts;
    P.ld_rowvec = a->ld_rowvec;
    P.h3_sa = std::ldexp(1.f, a->h3_exp_a);
    P.h3_sb = std::ldexp(1.f, a->h3_exp_b);
    P.h3_inv = std::ldexp(1.f, -(a->h3_exp_a + a->h3_exp_b));
    if (e == U2GNN_EPI_BIAS_DROP_RESID_LN) {   // N == 64: the tile rule above picked 64
        P.ln_gamma = a->ln_gamma;
        P.ln_beta = a->ln_beta;
        P.ln_y = a->ln_y;
        P.ln_ldy = a->ln_ldy;
        P.ln_mean = a->ln_mean;
        P.ln_rstd = a->ln_rstd;
        P.ln_d = (int32_t)a->ln_d;
        P.ln_rows = (int32_t)a->ln_rows;
        P.ln_eps = a->ln_eps;
    }
    G.P = P;
    G.tile = tile, G.split = split, G.prec = prec, G.epi = e;
    G.ta = a->trans_a != 0, G.tb = a->trans_b != 0, G.clamp = a->clamp_a != 0;
    return U2GNN_OK;
}

int gemm_launch(const u2gnn_gemm_args *a, GemmPlan &G, hipStream_t st) {
    if (G.prec == U2GNN_PREC_F16X3)
        return launch_tile<U2GNN_PREC_F16X3>(G.P, G.tile, G.ta, G.tb, G.epi, G.split, G.clamp, st);
    if (G.prec == U2GNN_PREC_BF16X6)
        return launch_tile<U2GNN_PREC_BF16X6>(G.P, G.tile, G.ta, G.tb, G.epi, G.split, G.clamp, st);
    if (G.prec == U2GNN_PREC_BF16X3)
        return launch_tile<U2GNN_PREC_BF16X3>(G.P, G.tile, G.ta, G.tb, G.epi, G.split, G.clamp, st);
    if (G.prec == U2GNN_PREC_BF16)
        return launch_tile<U2GNN_PREC_BF16>(G.P, G.tile, G.ta, G.tb, G.epi, G.split, G.clamp, st);
    return launch_tile<U2GNN_PREC_F32>(G.P, G.tile, G.ta, G.tb, G.epi, G.split, G.clamp, st);
}

// the grouped kernels: 64x64 and the 16-deep 128x128 (weight gradients), 256x128 (attention products)
template <int KIND>
int launch_group(GemmGroup &GG, int tile, int blocks, hipStream_t st) {
    constexpr bool SPLIT = KIND == U2GNN_PREC_BF16X3;
    if (tile == 64)
        hipLaunchKernelGGL((gemm_bf16_group_kernel<64, 64, 2, 2, 32, SPLIT>), dim3(blocks), dim3(256), 0, st, GG);
    else if (tile == 129)
        hipLaunchKernelGGL((gemm_bf16_group_kernel<128, 128, 2, 2, 16, SPLIT>), dim3(blocks), dim3(256), 0, st, GG);
    else
        hipLaunchKernelGGL((gemm_bf16_group_kernel<256, 128, 4, 2, 32, SPLIT>), dim3(blocks), dim3(512), 0, st, GG);
    return u2gnn_launch_status();
}

}  // namespace

extern "C" int u2gnn_gemm(const u2gnn_gemm_args *a, void *stream) {
    GemmPlan G;
    const int rc = gemm_plan(a, G);
    if (rc != U2GNN_OK) return rc;
    return gemm_launch(a, G, u2gnn_stream(stream));
}

extern "C" int u2gnn_gemm_group(const u2gnn_gemm_args *args, int32_t n, void *stream) {
    if (n < 0 || n > GG_MAX || (n && !args)) return U2GNN_E_ARG;
    hipStream_t st = u2gnn_stream(stream);
    GemmPlan G[GG_MAX];
    for (int32_t i = 0; i < n; ++i) {
        const int rc = gemm_plan(&args[i], G[i]);
        if (rc != U2GNN_OK) return rc;
    }
    // one launch when every job runs the same grouped kernel
    bool same = n > 1;
    for (int32_t i = 0; i < n && same; ++i)
        same = G[i].prec == G[0].prec && G[i].prec != U2GNN_PREC_F32 && !fwd_kind(G[i].prec) &&
               G[i].tile == G[0].tile &&
               (G[i].tile == 64 || G[i].tile == 129 || G[i].tile == 256) && !G[i].tb && G[i].epi == U2GNN_EPI_STORE &&
               (G[i].ta || !G[i].clamp);
    if (!same) {
        for (int32_t i = 0; i < n; ++i) {
            const int rc = gemm_launch(&args[i], G[i], st);
            if (rc != U2GNN_OK) return rc;
        }
        return U2GNN_OK;
    }
    GemmGroup GG;
    std::memset(&GG, 0, sizeof(GG));
    GG.n = n;
    int64_t blocks = 0;
    for (int32_t i = 0; i < n; ++i) {
        GG.p[i] = G[i].P;
        GG.layout[i] = !G[i].ta ? GG_NN : (G[i].clamp ? GG_TA_CLAMP : GG_TA);
        GG.start[i] = (int32_t)blocks;
        blocks += (int64_t)G[i].P.gm * G[i].P.gn * G[i].split;
    }
    if (blocks >= ((int64_t)1 << 31)) return U2GNN_E_SHAPE;
    GG.start[n] = (int32_t)blocks;
    if (G[0].prec == U2GNN_PREC_BF16X3) return launch_group<U2GNN_PREC_BF16X3>(GG, G[0].tile, (int)blocks, st);
    return launch_group<U2GNN_PREC_BF16>(GG, G[0].tile, (int)blocks, st);
}
