// bf16x3 GEMM over pre-split operands (x2 format, include/u2gnn_hip.h) for the six N^2 attention
// products of the U2GNN encoder: S = Q.K^T, O = Pd.V, dS = dO.V^T (+ recomputed-P epilogue),
// dV = Pd^T.dO, dQ = dS.K, dK = dS^T.Q (torch MultiheadAttention inside the reference's
// TransformerEncoderLayer, pytorch_U2GNN_Sup.py:19-21,35 / pytorch_U2GNN_UnSup.py:37-40,57).
//
// Why a second kernel: the fp32-operand BF16X3 kernel (gemm.hip) splits every operand into hi/lo
// bf16 while staging it through registers, one barrier per K step; measured there, the staging
// (global->register->split->LDS) and not the matrix pipe bounds it at ~35 % of the MFMA rate.  Here
// the producers (QKV projection epilogue, softmax, dO and dS epilogues) write the operands already
// split, so staging is a pure copy, done by LDS-DMA (global_load_lds_dwordx4: no VGPRs, no VALU, no
// ds_write):
//   * 3-stage LDS ring, tiles t+1 and t+2 in flight while tile t is multiplied; one raw s_barrier
//     per K step preceded by a counted vmcnt (never 0 inside the loop) — __syncthreads() would
//     drain the DMA queue;
//   * LDS images are lane-linear (an LDS-DMA writes base + 16*lane), so the bank swizzles live on
//     the per-lane SOURCE address and the matching XOR on the fragment reads:
//       [rows][K] operands: 128-B rows (32 k of hi+lo), 16-B chunk q stored at q ^ ((row>>1)&7)
//         -> conflict-free ds_read_b128 fragment reads;
//       [K][rows] operands: 4*R-byte k-rows, byte ^= ((k&1)<<4) | ((k&2)<<6)
//         -> conflict-free ds_read_b64_tr_b16 fragment reads;
//   * 8 waves (4x2) on 256x128 blocks or 4 waves (2x2) on 128x128, 64x64 per wave, 32x32x16 MFMAs
//     in the same order as gemm.hip (bh*al, bl*ah, bh*ah), so results are bit-identical to it;
//   * the epilogues of gemm_common.h (fp32 and/or x2 output, split-K slabs).
#include "gemm_common.h"

namespace {



typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((address_space(3))) void lds_void;

// image bytes of one operand tile with R rows (either layout): R * BK k * 2 planes * 2 B
template <int R, int BK> constexpr int img_bytes() { return R * BK * 4; }
// RK row swizzle: 16-B chunk q of row r is stored at q ^ rk_swz(r); rows are BK*4 bytes (8 or 4 chunks),
// chosen so that every 16-lane group of a ds_read_b128 fragment read hits 16 distinct bank slots
template <int BK> __device__ __forceinline__ int rk_swz(int r) { return BK == 32 ? (r >> 1) & 7 : (r >> 2) & 3; }

__device__ __forceinline__ int kr_swz(int krow) { return ((krow & 1) << 4) | ((krow & 2) << 6); }

// Per-lane source byte offsets of the NI LDS-DMA instructions that fill one tile of an operand
// with R rows.  Instruction i of wave w writes image bytes [(i*NT + 64w)*16, +1024).
//   RK (operand stored [rows][K]): chunk c -> row c/8, stored chunk position c%8 holds logical chunk
//     q = (c%8) ^ ((row>>1)&7) = k-group q/2, plane q%2 -> source row*ld + q/2*32 B + (q%2)*16 B.
//   KR (operand stored [K][rows]): byte 16c -> k-row 16c/(4R), position p -> logical byte
//     p ^ kr_swz(k-row) -> source k-row*ld + col0*4 B + logical byte.
template <int R, int BK, bool KR, int NT>
__device__ __forceinline__ void x2_src_init(int tid, int64_t ld_bytes, int64_t (&off)[img_bytes<R, BK>() / (16 * NT)]) {
    constexpr int NI = img_bytes<R, BK>() / (16 * NT), NCH = BK / 4;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int c = i * NT + tid;
        if constexpr (!KR) {
            const int r = c / NCH, q = (c % NCH) ^ rk_swz<BK>(r);
            off[i] = (int64_t)r * ld_bytes + (q >> 1) * 32 + (q & 1) * 16;
        } else {
            const int b = c * 16, kr = b / (4 * R), p = b % (4 * R);
            off[i] = (int64_t)kr * ld_bytes + (p ^ kr_swz(kr));
        }
    }
}

template <int NI, int NT>
__device__ __forceinline__ void x2_issue(const char *src, const int64_t (&off)[NI], char *img, int w) {
#pragma unroll
    for (int i = 0; i < NI; ++i)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(src + off[i]),
                                         (lds_void *)(img + (i * NT + 64 * w) * 16), 16, 0, 0);
}

// MFMA operand fragment (32 rows x 16 k, lane l: row r0 + l%32, k = ks*16 + 8*(l/32) .. +7), hi and lo
template <int R, int BK, bool KR>
__device__ __forceinline__ void x2_frag(const char *img, int r0, int ks, int lane, bf16x8 &hi, bf16x8 &lo) {
    if constexpr (!KR) {
        const int r = r0 + (lane & 31), gk = 2 * ks + (lane >> 5), sw = rk_swz<BK>(r);
        const char *row = img + r * (BK * 4);
        hi = *reinterpret_cast<const bf16x8 *>(row + (((2 * gk) ^ sw) << 4));
        lo = *reinterpret_cast<const bf16x8 *>(row + (((2 * gk + 1) ^ sw) << 4));
    } else {
        // ds_read_b64_tr_b16: in each 16-lane group, lane 4q+p supplies k-row q, columns 4p..4p+3 of a
        // 4 x 16 block and receives column (lane % 16) of the 4 k-rows
        const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
        const int kr = ks * 16 + (g >> 1) * 8 + q;
        const int col = r0 + (g & 1) * 16 + 4 * p;               // 4 consecutive columns, one 8-group half
        const int cb = (col >> 3) * 32 + (col & 7) * 2;           // hi byte inside the k-row
        // kr + 4 has the same swizzle; the lo plane is 16 B further in LOGICAL bytes (cb has bit 4
        // clear, the swizzle may set it: XOR after the offset, never add to the swizzled address)
        const char *a = img + kr * (4 * R) + (cb ^ kr_swz(kr));
        const char *b = img + kr * (4 * R) + ((cb + 16) ^ kr_swz(kr));
        const s16x4 h0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(a));
        const s16x4 h1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(a + 16 * R));
        const s16x4 l0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(b));
        const s16x4 l1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(b + 16 * R));
        const s16x4 vh[2] = {h0, h1}, vl[2] = {l0, l1};
        hi = __builtin_bit_cast(bf16x8, vh);
        lo = __builtin_bit_cast(bf16x8, vl);
    }
}

template <int N_>
__device__ __forceinline__ void wait_vm() {
    if constexpr (N_ == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if constexpr (N_ == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else if constexpr (N_ == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if constexpr (N_ == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if constexpr (N_ == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if constexpr (N_ == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else if constexpr (N_ == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else static_assert(N_ == 0, "add the vmcnt literal");
}

template <int BM, int BN, int WM, int WN, int BK, int NS, int MINB, bool PP, bool TA, bool TB, int EPI>
__global__ void __launch_bounds__(64 * WM * WN, MINB) gemm_x2_kernel(GemmP P) {
    if constexpr (EPI == U2GNN_EPI_BIAS_DROP_RESID || EPI == U2GNN_EPI_BIAS_RELU_DROP || EPI == U2GNN_EPI_ATTN_DS_RECOMP)
        P.seed = u2gnn_seed(P.seed, P.epoch);   // graph replay: device-resident seed epoch
    constexpr int NT = 64 * WM * WN;
    constexpr int WTM = BM / WM, WTN = BN / WN;        // wave tile
    constexpr int TM = WTM / 32, TN = WTN / 32;
    constexpr bool KRA = TA, KRB = !TB;                // which operands are stored [K][rows]
    constexpr int AB = img_bytes<BM, BK>(), BB = img_bytes<BN, BK>(), STAGE = AB + BB;
    constexpr int NIA = AB / (16 * NT), NIB = BB / (16 * NT), NI = NIA + NIB;
    static_assert(NIA * 16 * NT == AB && NIB * 16 * NT == BB, "tile not a multiple of the DMA footprint");
    static_assert(NS == 2 || NS == 3, "2 or 3 LDS stages");
    static_assert(!PP || (NS == 3 && WM * WN == 8), "ping-pong: 8 waves, 3 stages");
    __shared__ __attribute__((aligned(1024))) char smem[NS * STAGE];

    const int tid = threadIdx.x;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63;
    int tmi, tni, zi;
    tile_coords(P.gm, P.gn, tmi, tni, zi);
    const int m0 = tmi * BM, n0 = tni * BN;
    const int64_t kbase = (int64_t)zi * P.K;
    const int64_t klen = min((int64_t)P.K, (int64_t)P.Ktot - kbase);
    const int nk = klen > 0 ? (int)(klen / BK) : 0;

    // operand tile origins (bytes); one K step advances RK images by BK*4 B, KR images by BK k-rows
    const int64_t ldaB = P.lda * 2, ldbB = P.ldb * 2;
    const char *Ab = reinterpret_cast<const char *>(P.A2) +
                     (KRA ? kbase * ldaB + (int64_t)m0 * 4 : (int64_t)m0 * ldaB + kbase * 4);
    const char *Bb = reinterpret_cast<const char *>(P.B2) +
                     (KRB ? kbase * ldbB + (int64_t)n0 * 4 : (int64_t)n0 * ldbB + kbase * 4);
    const int64_t stepA = KRA ? BK * ldaB : BK * 4;
    const int64_t stepB = KRB ? BK * ldbB : BK * 4;
    int64_t offA[NIA], offB[NIB];
    x2_src_init<BM, BK, KRA, NT>(tid, ldaB, offA);
    x2_src_init<BN, BK, KRB, NT>(tid, ldbB, offB);

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int wm = w / WN, wn = w % WN;
    auto issue = [&](int kt, int s) {
        char *img = smem + s * STAGE;
        x2_issue<NIA, NT>(Ab + kt * stepA, offA, img, w);
        x2_issue<NIB, NT>(Bb + kt * stepB, offB, img + AB, w);
    };
    auto compute = [&](const char *img) {
        const char *Ai = img, *Bi = img + AB;
#pragma unroll
        for (int ks = 0; ks < BK / 16; ++ks) {
            bf16x8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) x2_frag<BM, BK, KRA>(Ai, wm * WTM + i * 32, ks, lane, ah[i], al[i]);
#pragma unroll
            for (int j = 0; j < TN; ++j) x2_frag<BN, BK, KRB>(Bi, wn * WTN + j * 32, ks, lane, bh[j], bl[j]);
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bh[j], al[i], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bl[j], ah[i], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bh[j], ah[i], acc[i][j], 0, 0, 0);
                }
        }
    };

    if constexpr (PP) {
        // Ping-pong schedule: waves 0-3 and 4-7 (one of each on every SIMD) run the same
        // load-phase / MFMA-phase loop one barrier apart, so each SIMD's matrix pipe alternates
        // between its two waves while the other one reads its next fragments.  Per K step t:
        //   load phase: issue tile t+2 (stage (t+2)%3, last read as tile t-1), ds_read all of
        //               tile t, wait for this thread's DMA of tile t+1 and its own LDS reads, barrier
        //   MFMA phase: 3 x TM x TN x BK/16 MFMAs at raised priority, barrier
        // Hazards (global barrier index: group 0 code barrier c = global c, group 1 = c + 1):
        //   RAW  tile t+1 is first read after global 2t+2; every thread waited for its share of it
        //        before global 2t+1 (group 0) / 2t+2 (group 1)
        //   WAR  tile t-1 reads completed (lgkmcnt(0)) before global 2t-1 / 2t; stage (t-1)%3 is
        //        restaged after global 2t / 2t+1
        const bool g1 = w >= 4;
        if (0 < nk) issue(0, 0);
        if (1 < nk) issue(1, 1);
        if (1 < nk) wait_vm<NI>();
        else wait_vm<0>();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (g1) {
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
        }
        for (int t = 0; t < nk; ++t) {
            if (t + 2 < nk) issue(t + 2, (t + 2) % 3);
            const char *Ai = smem + (t % 3) * STAGE, *Bi = Ai + AB;
            bf16x8 ah[BK / 16][TM], al[BK / 16][TM], bh[BK / 16][TN], bl[BK / 16][TN];
#pragma unroll
            for (int ks = 0; ks < BK / 16; ++ks) {
#pragma unroll
                for (int i = 0; i < TM; ++i) x2_frag<BM, BK, KRA>(Ai, wm * WTM + i * 32, ks, lane, ah[ks][i], al[ks][i]);
#pragma unroll
                for (int j = 0; j < TN; ++j) x2_frag<BN, BK, KRB>(Bi, wn * WTN + j * 32, ks, lane, bh[ks][j], bl[ks][j]);
            }
            if (t + 2 < nk) wait_vm<NI>();
            else wait_vm<0>();
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int ks = 0; ks < BK / 16; ++ks)
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j) {
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bh[ks][j], al[ks][i], acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bl[ks][j], ah[ks][i], acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bh[ks][j], ah[ks][i], acc[i][j], 0, 0, 0);
                    }
            __builtin_amdgcn_s_setprio(0);
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
        }
        if (!g1) __builtin_amdgcn_s_barrier();   // same barrier count in both groups
    } else {
#pragma unroll
    for (int s = 0; s < NS - 1; ++s)
        if (s < nk) issue(s, s);
    for (int t = 0; t < nk; ++t) {
        // this thread's DMA for tile t has landed (with 3 stages tile t+1 may still be in flight);
        // after the barrier every thread's has, and every wave is done reading stage (t-1)%NS
#ifndef X2_EXP_NOSYNC
        if (NS == 3 && t + 1 < nk) wait_vm<NI>();
        else wait_vm<0>();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
#endif
#ifndef X2_EXP_NOLOAD
        if (t + NS - 1 < nk) issue(t + NS - 1, (t + NS - 1) % NS);
#endif
        compute(smem + (t % NS) * STAGE);
    }
    }
#ifdef X2_EXP_NOSYNC
    wait_vm<0>();
#endif
#ifdef X2_EXP_NOEPI
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) asm volatile("" ::"v"(acc[i][j]));
    return;
#endif

    store_tile<EPI>(P, P.C ? P.C + (int64_t)zi * P.slab_stride : nullptr, acc, m0 + wm * WTM, n0 + wn * WTN,
                    lane & 31, lane >> 5, (const PreDS<TN> *)nullptr);
}

// tile codes (u2gnn_gemm_args.tile) of the x2 kernel:
//   256: 256x128, BK 32, 3 stages (144 KB LDS, 1 block/CU)    257: 256x128, BK 16, 3 stages (72 KB, 2 blocks/CU)
//   128: 128x128, BK 16, 3 stages (48 KB, 3 blocks/CU)        130: 128x128, BK 32, 2 stages (64 KB, 2 blocks/CU)
//   258: 256x128, 4 waves of 128x64, BK 16, 3 stages (72 KB, 2 blocks/CU)
//   259: 256x128, 4 waves of 128x64, BK 32, 2 stages (96 KB, 1 block/CU)
//   260: 256x256, 8 waves of 128x64, BK 16, 3 stages (96 KB, 1 block/CU)
//   261 / 262 / 263: the ping-pong schedule (PP) on 256x128 BK 32, 256x256 BK 16, 256x128 BK 16
template <int CODE> struct X2Cfg;
template <> struct X2Cfg<256> { static constexpr int BM = 256, BN = 128, WM = 4, WN = 2, BK = 32, NS = 3, MINB = 1; static constexpr bool PP = false; };
template <> struct X2Cfg<257> { static constexpr int BM = 256, BN = 128, WM = 4, WN = 2, BK = 16, NS = 3, MINB = 2; static constexpr bool PP = false; };
template <> struct X2Cfg<128> { static constexpr int BM = 128, BN = 128, WM = 2, WN = 2, BK = 16, NS = 3, MINB = 3; static constexpr bool PP = false; };
template <> struct X2Cfg<130> { static constexpr int BM = 128, BN = 128, WM = 2, WN = 2, BK = 32, NS = 2, MINB = 2; static constexpr bool PP = false; };
template <> struct X2Cfg<258> { static constexpr int BM = 256, BN = 128, WM = 2, WN = 2, BK = 16, NS = 3, MINB = 2; static constexpr bool PP = false; };
template <> struct X2Cfg<259> { static constexpr int BM = 256, BN = 128, WM = 2, WN = 2, BK = 32, NS = 2, MINB = 1; static constexpr bool PP = false; };
template <> struct X2Cfg<260> { static constexpr int BM = 256, BN = 256, WM = 2, WN = 4, BK = 16, NS = 3, MINB = 1; static constexpr bool PP = false; };
template <> struct X2Cfg<261> { static constexpr int BM = 256, BN = 128, WM = 4, WN = 2, BK = 32, NS = 3, MINB = 1; static constexpr bool PP = true; };
template <> struct X2Cfg<262> { static constexpr int BM = 256, BN = 256, WM = 2, WN = 4, BK = 16, NS = 3, MINB = 1; static constexpr bool PP = true; };
template <> struct X2Cfg<263> { static constexpr int BM = 256, BN = 128, WM = 4, WN = 2, BK = 16, NS = 3, MINB = 1; static constexpr bool PP = true; };

template <int CODE, bool TA, bool TB>
int x2_launch_epi(const GemmP &P, int epi, int split, hipStream_t st) {
    using C = X2Cfg<CODE>;
    constexpr int NT = 64 * C::WM * C::WN;
    const dim3 grid(P.gm * P.gn * split), block(NT);
    switch (epi) {
        case U2GNN_EPI_STORE:
            hipLaunchKernelGGL((gemm_x2_kernel<C::BM, C::BN, C::WM, C::WN, C::BK, C::NS, C::MINB, C::PP, TA, TB, U2GNN_EPI_STORE>), grid, block,
                               0, st, P);
            break;
        case U2GNN_EPI_ATTN_DS_RECOMP:
            if constexpr (!TA && TB) {
                hipLaunchKernelGGL((gemm_x2_kernel<C::BM, C::BN, C::WM, C::WN, C::BK, C::NS, C::MINB, C::PP, TA, TB, U2GNN_EPI_ATTN_DS_RECOMP>),
                                   grid, block, 0, st, P);
                break;
            } else {
                return U2GNN_E_ARG;
            }
        default: return U2GNN_E_ARG;
    }
    return u2gnn_launch_status();
}

template <int CODE>
int x2_launch_layout(const GemmP &P, bool ta, bool tb, int epi, int split, hipStream_t st) {
    if (!ta && tb) return x2_launch_epi<CODE, false, true>(P, epi, split, st);
    if (!ta && !tb) return x2_launch_epi<CODE, false, false>(P, epi, split, st);
    if (ta && !tb) return x2_launch_epi<CODE, true, false>(P, epi, split, st);
    return U2GNN_E_ARG;
}

inline bool al16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

// called by u2gnn_gemm (gemm.hip) when a_x2 / b_x2 are set; P already holds every common field
int u2gnn_gemm_x2_dispatch(const u2gnn_gemm_args *a, GemmP &P, int tile, int split, hipStream_t st) {
    if (a->precision != U2GNN_PREC_BF16X3 || !a->a_x2 || !a->b_x2 || !a->A2 || !a->B2) return U2GNN_E_ARG;
    if (tile != 256 && tile != 257 && tile != 128 && tile != 130 && (tile < 258 || tile > 263)) return U2GNN_E_ARG;
    if (a->clamp_a) return U2GNN_E_ARG;
    if (!al16(a->A2) || !al16(a->B2) || (a->lda & 15) || (a->ldb & 15)) return U2GNN_E_ALIGN;
    const int bk = (tile == 256 || tile == 130 || tile == 259 || tile == 261) ? 32 : 16;
    if (a->K % bk) return U2GNN_E_SHAPE;
    // DMA sources are 64-bit per-lane pointers: no 32-bit offset limit, but rows must lie inside the
    // operand: the caller guarantees M, N, K multiples of the tile (checked by u2gnn_gemm)
    const int bm = tile >= 256 ? 256 : 128, bn = (tile == 260 || tile == 262) ? 256 : 128;
    if (a->M % bm || a->N % bn) return U2GNN_E_SHAPE;
    P.gm = (int32_t)(a->M / bm);
    P.gn = (int32_t)(a->N / bn);
    // split-K granule = the kernel's K step
    P.K = (int32_t)((a->K + (int64_t)split * bk - 1) / ((int64_t)split * bk) * bk);
    const bool ta = a->trans_a != 0, tb = a->trans_b != 0;
    if (tile == 256) return x2_launch_layout<256>(P, ta, tb, a->epilogue, split, st);
    if (tile == 257) return x2_launch_layout<257>(P, ta, tb, a->epilogue, split, st);
    if (tile == 130) return x2_launch_layout<130>(P, ta, tb, a->epilogue, split, st);
    if (tile == 258) return x2_launch_layout<258>(P, ta, tb, a->epilogue, split, st);
    if (tile == 259) return x2_launch_layout<259>(P, ta, tb, a->epilogue, split, st);
    if (tile == 260) return x2_launch_layout<260>(P, ta, tb, a->epilogue, split, st);
    if (tile == 261) return x2_launch_layout<261>(P, ta, tb, a->epilogue, split, st);
    if (tile == 262) return x2_launch_layout<262>(P, ta, tb, a->epilogue, split, st);
    if (tile == 263) return x2_launch_layout<263>(P, ta, tb, a->epilogue, split, st);
    return x2_launch_layout<128>(P, ta, tb, a->epilogue, split, st);
}
