// bf16x3 GEMM over pre-split (x2) operands with 16x16x32 MFMAs, persistent over output tiles, with
// a ping-pong wave schedule — the N^2 attention products of the U2GNN encoder whose operands are
// both stored [rows][K] (S = Q.K^T, dS = dO.V^T with the signed-image epilogue; torch
// MultiheadAttention inside pytorch_U2GNN_Sup.py:19-21,35).  Both have a short K (d = 367 -> 384)
// and an N^2 output, so one block stays resident per CU and the stores of tile i drain under tile
// i+1's K loop.
//
// Geometry: 256x128 blocks, 8 waves (4 x 2) of 64x64, 16x16 MFMA blocks; a K tile is 32 real k =
// 64 bf16 per row (hi/lo planes interleaved per 8 k: the x2 format), i.e. 128-B LDS rows; each block
// takes three MFMAs per K tile (bh*al, bl*ah, bh*ah).  Three 48-KB LDS stages.
// Staging: global_load_lds_dwordx4 (LDS-DMA: no VGPRs, no VALU, no ds_write); the image is
// lane-linear, so the bank swizzle is applied to the per-lane SOURCE chunk and the same XOR on the
// reads (cdna_hip_programming.md §5.4 rule 21): chunk c of row r sits at c ^ x3_swz(r % 16),
// conflict-free for every ds_read_b128 lane group of a 16x16x32 fragment read (exhaustive check:
// DESIGN.md §5.3).
// Ping-pong (cdna_hip_programming.md §5, 8-phase template, its wave-group stagger): waves 0-3 and
// 4-7 (one of each on every SIMD) run the same loop one barrier apart, so while one group runs its
// 48 MFMAs per K tile the other reads its 16 fragments; hardware barrier H(2t) = group-0 barrier_a
// of K tile t, H(2t+1) = group-0 barrier_b = group-1 barrier_a, H(2t+2) = group-1 barrier_b.
//   LOAD(t):  wait for this thread's DMA of tile t+1 (issued one iteration earlier), ds_read tile t
//   barrier_a; lgkmcnt(0); DMA of tile t+2 into stage (t+2)%3; MFMA(t) at raised priority; barrier_b
// Hazards: RAW tile t+1 is first read by group 0 after H(2t+1); group 0 waited for its share before
//   H(2t), group 1 before H(2t+1).  WAR stage (t+2)%3 = (t-1)%3: group 0 finished its reads of t-1
//   before H(2t-1), group 1 before H(2t); the DMA is issued after H(2t) (group 0) / H(2t+1).
// K tiles are counted across the block's output tiles, so the DMA two tiles ahead may already belong
// to the next output tile; after an epilogue the wait is vmcnt(NSTORE) (the stores are younger than
// the DMA and stay in flight).
#include "gemm_common.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void3;

constexpr int X3_NT = 512;
constexpr int X3_ROWB = 128;   // bytes per image row: 32 k x (hi + lo) x 2 B
constexpr int X3_BM = 256, X3_BN = 128;
constexpr int X3_A_IMG = X3_BM * X3_ROWB, X3_B_IMG = X3_BN * X3_ROWB, X3_STAGE = X3_A_IMG + X3_B_IMG;
constexpr int X3_NS = 3;
constexpr int X3_NIA = X3_BM / 64, X3_NIB = X3_BN / 64;   // DMA instructions per thread per K tile

// 16-B chunk c of image row r sits at position c ^ x3_swz(r % 16)
__device__ __forceinline__ int x3_swz(int r) { return ((r >> 1) & 7) ^ ((((r >> 2) ^ (r >> 3)) & 1) << 1); }

// Per-lane source byte offsets of the LDS-DMA instructions that fill an R-row image of an operand
// stored [rows][K] in x2 format.  Instruction i of wave w writes image bytes [(8i + w) KB, +1 KB)
// = rows 64i + 8w .. +7; lane L fills row 64i + 8w + L/8 at position L%8, which holds logical
// chunk (L%8) ^ x3_swz(row).
template <int R>
__device__ __forceinline__ void x3_src_init(int w, int lane, int64_t ld_bytes, int64_t (&off)[R / 64]) {
#pragma unroll
    for (int i = 0; i < R / 64; ++i) {
        const int r = 64 * i + 8 * w + (lane >> 3);
        const int c = (lane & 7) ^ x3_swz(r & 15);
        off[i] = (int64_t)r * ld_bytes + c * 16;
    }
}

template <int NI>
__device__ __forceinline__ void x3_issue(const char *src, const int64_t (&off)[NI], char *img, int w) {
#pragma unroll
    for (int i = 0; i < NI; ++i)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(src + off[i]),
                                         (lds_void3 *)(img + (8 * i + w) * 1024), 16, 0, 0);
}

// 16x16x32 fragment (lane l: row r0 + l%16, k = 8*(l/16) .. +7) of plane p (0 hi, 1 lo)
__device__ __forceinline__ bf16x8 x3_frag(const char *img, int r0, int lane, int p) {
    const int r = r0 + (lane & 15);
    const int c = 2 * (lane >> 4) + p;
    return *reinterpret_cast<const bf16x8 *>(img + r * X3_ROWB + ((c ^ x3_swz(lane & 15)) << 4));
}

template <int N_>
__device__ __forceinline__ void x3_wait_vm() {
    static_assert(N_ >= 0 && N_ < 64, "vmcnt range");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N_) : "memory");
}

__device__ __forceinline__ void x3_barrier() {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// logical tile L -> (tm, tn): groups of 8 row tiles, row tile fastest inside a group (blocks that
// run at the same time on one XCD share A row panels and B column panels in its L2)
__device__ __forceinline__ void x3_tile(int L, int gm, int gn, int &tm, int &tn) {
    constexpr int GROUP = 8;
    const int per_group = GROUP * gn;
    const int g = L / per_group;
    const int first_m = g * GROUP;
    const int gsz = min(gm - first_m, GROUP);
    const int in_g = L - g * per_group;
    tm = first_m + in_g % gsz;
    tn = in_g / gsz;
}

template <int EPI>
__global__ void __launch_bounds__(X3_NT) gemm_x3_nt_kernel(GemmP P) {
    if constexpr (EPI == U2GNN_EPI_BIAS_DROP_RESID || EPI == U2GNN_EPI_BIAS_RELU_DROP || EPI == U2GNN_EPI_ATTN_DS_RECOMP)
        P.seed = u2gnn_seed(P.seed, P.epoch);   // graph replay: device-resident seed epoch
    constexpr int WN = 2, WTM = 64, WTN = 64, MB = 4, NB = 4;
    constexpr int NSTORE = MB * NB;   // float4 stores per thread per output tile
    __shared__ __attribute__((aligned(1024))) char smem[X3_NS * X3_STAGE];

    const int tid = threadIdx.x;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63;
    const int wm = w / WN, wn = w % WN;
    const bool g1 = w >= 4;   // ping-pong group (waves w and w + 4 share a SIMD)
    const int ntile = P.gm * P.gn;
    const int nk = P.K / 32;
    // persistent: logical tiles wgid, wgid + G, ...; wgid = XCD-contiguous remap of blockIdx
    const int G = (int)gridDim.x;
    const int q = G >> 3, r8 = G & 7, xcd = (int)blockIdx.x & 7, loc = (int)blockIdx.x >> 3;
    const int wgid = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + loc;
    if (wgid >= ntile || nk == 0) return;
    const int ntiles_mine = (ntile - wgid + G - 1) / G;
    const int total = ntiles_mine * nk;   // K tiles this block runs

    const int64_t ldaB = P.lda * 2, ldbB = P.ldb * 2;
    int64_t offA[X3_NIA], offB[X3_NIB];
    x3_src_init<X3_BM>(w, lane, ldaB, offA);
    x3_src_init<X3_BN>(w, lane, ldbB, offB);
    const char *A2 = reinterpret_cast<const char *>(P.A2);
    const char *B2 = reinterpret_cast<const char *>(P.B2);

    // DMA of this block's K tile number u (u = tile_index * nk + kt) into stage u % 3
    auto issue = [&](int u) {
        const int L = wgid + (u / nk) * G, kt = u % nk;
        int tm, tn;
        x3_tile(L, P.gm, P.gn, tm, tn);
        char *img = smem + (u % X3_NS) * X3_STAGE;
        x3_issue<X3_NIA>(A2 + (int64_t)tm * X3_BM * ldaB + kt * X3_ROWB, offA, img, w);
        x3_issue<X3_NIB>(B2 + (int64_t)tn * X3_BN * ldbB + kt * X3_ROWB, offB, img + X3_A_IMG, w);
    };

    f32x4 acc[MB][NB];
#pragma unroll
    for (int i = 0; i < MB; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    issue(0);
    if (total > 1) {
        issue(1);
        x3_wait_vm<X3_NIA + X3_NIB>();
    } else {
        x3_wait_vm<0>();
    }
    x3_barrier();
    if (g1) x3_barrier();
    const int li = lane & 15, cq = 4 * (lane >> 4);
    bool after_epi = false;
    for (int u = 0; u < total; ++u) {
        const int kt = u % nk;
        // LOAD(u): this thread's DMA of K tile u+1 (older than any epilogue store)
        if (after_epi) x3_wait_vm<NSTORE>();
        else x3_wait_vm<0>();
        after_epi = false;
        const char *Ai = smem + (u % X3_NS) * X3_STAGE, *Bi = Ai + X3_A_IMG;
        bf16x8 ah[MB], al[MB], bh[NB], bl[NB];
#pragma unroll
        for (int i = 0; i < MB; ++i) {
            ah[i] = x3_frag(Ai, wm * WTM + i * 16, lane, 0);
            al[i] = x3_frag(Ai, wm * WTM + i * 16, lane, 1);
        }
#pragma unroll
        for (int j = 0; j < NB; ++j) {
            bh[j] = x3_frag(Bi, wn * WTN + j * 16, lane, 0);
            bl[j] = x3_frag(Bi, wn * WTN + j * 16, lane, 1);
        }
        x3_barrier();   // barrier_a
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
#ifndef X3_EXP_NOLOAD   // experiment: no DMA after the prologue (compute + ds_read bound)
        if (u + 2 < total) issue(u + 2);
#endif
        __builtin_amdgcn_s_setprio(1);
#ifdef X3_EXP_NOMFMA   // experiment: no MFMAs (staging bound)
#pragma unroll
        for (int i = 0; i < MB; ++i) asm volatile("" ::"v"(ah[i]), "v"(al[i]));
#pragma unroll
        for (int j = 0; j < NB; ++j) asm volatile("" ::"v"(bh[j]), "v"(bl[j]));
        if (false)
#endif
#pragma unroll
        for (int i = 0; i < MB; ++i)
#pragma unroll
            for (int j = 0; j < NB; ++j) {
                // B fragment first: the accumulator holds the tile transposed (lane: one row, 4
                // consecutive columns -> 16-byte epilogue accesses)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh[j], al[i], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bl[j], ah[i], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh[j], ah[i], acc[i][j], 0, 0, 0);
            }
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        x3_barrier();   // barrier_b
        if (kt == nk - 1) {
            // epilogue: lane holds C[row = r0 + lane%16][cols c0 + 4*(lane/16) .. +3] of each block
            int tm, tn;
            x3_tile(wgid + (u / nk) * G, P.gm, P.gn, tm, tn);
            const int m0 = tm * X3_BM + wm * WTM, n0 = tn * X3_BN + wn * WTN;
#pragma unroll
            for (int i = 0; i < MB; ++i) {
                const int row = m0 + i * 16 + li;
                float4 a[NB], b[NB];
                uint32_t kb[NB];
                const float dl = (EPI == U2GNN_EPI_ATTN_DS_SIGNED) ? P.rowvec[row] : 0.f;
#pragma unroll
                for (int j = 0; j < NB; ++j) {
                    a[j] = b[j] = make_float4(0.f, 0.f, 0.f, 0.f);
                    kb[j] = 0;
                    epi_fetch<EPI>(P, row, n0 + j * 16 + cq, a[j], b[j], kb[j]);
                }
#pragma unroll
                for (int j = 0; j < NB; ++j) {
                    const int col = n0 + j * 16 + cq;
                    const f32x4 v = acc[i][j];
                    const float4 o =
                        epilogue4<EPI>(P, row, col, make_float4(v[0], v[1], v[2], v[3]), a[j], b[j], kb[j], dl);
                    *reinterpret_cast<float4 *>(P.C + (int64_t)row * P.ldc + col) = o;
                    acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
                }
            }
            after_epi = true;
        }
    }
    if (!g1) x3_barrier();   // same barrier count in both groups
}

template <int EPI>
int x3_launch(const GemmP &P, hipStream_t st) {
    const int tiles = P.gm * P.gn;
    const dim3 grid(tiles < 256 ? tiles : 256), block(X3_NT);   // one resident block per CU
    hipLaunchKernelGGL(gemm_x3_nt_kernel<EPI>, grid, block, 0, st, P);
    return u2gnn_launch_status();
}

}  // namespace

// tile code 301 of u2gnn_gemm: x2 operands, NT layout, fp32 C, STORE or ATTN_DS_SIGNED epilogue,
// no split-K, M % 256 == 0, N % 128 == 0, K % 32 == 0
int u2gnn_gemm_x3_dispatch(const u2gnn_gemm_args *a, GemmP &P, int tile, int split, hipStream_t st) {
    if (a->precision != U2GNN_PREC_BF16X3 || !a->a_x2 || !a->b_x2 || !a->A2 || !a->B2 || !a->C || a->Cx2)
        return U2GNN_E_ARG;
    if (tile != 301 || a->trans_a || !a->trans_b || a->clamp_a || split != 1) return U2GNN_E_ARG;
    if ((reinterpret_cast<uintptr_t>(a->A2) & 15) || (reinterpret_cast<uintptr_t>(a->B2) & 15) || (a->lda & 15) ||
        (a->ldb & 15))
        return U2GNN_E_ALIGN;
    if (a->K % 32 || a->M % X3_BM || a->N % X3_BN) return U2GNN_E_SHAPE;
    P.gm = (int32_t)(a->M / X3_BM);
    P.gn = (int32_t)(a->N / X3_BN);
    P.K = (int32_t)a->K;
    switch (a->epilogue) {
        case U2GNN_EPI_STORE: return x3_launch<U2GNN_EPI_STORE>(P, st);
        case U2GNN_EPI_ATTN_DS_SIGNED: return x3_launch<U2GNN_EPI_ATTN_DS_SIGNED>(P, st);
        default: return U2GNN_E_ARG;
    }
}
