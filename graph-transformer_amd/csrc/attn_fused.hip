// Attention forward over the node axis after S = Q K^T (a3.2 of SURVEY.md §8: softmax(Q K^T) -> dropout ->
// . V inside torch's MultiheadAttention, pytorch_U2GNN_Sup.py:19-21,35 / pytorch_U2GNN_UnSup.py:37-40,57).
//
// The scores come from the QK^T GEMM, whose epilogue also leaves per-row softmax partials
// (EPI_STORE_ROWSTAT, per 64-column group; masked keys stored as -inf); one fused kernel folds those
// into (max, 1/sum) per row and then does what the softmax pass and the P.V GEMM did: it reads each
// score once, forms P = exp(s - max)/sum and the dropout decision in registers, writes the signed
// image the backward reads (the only N x N write left in the forward) and multiplies the kept
// probabilities into V on the matrix cores (split bf16, 3 products per term) without staging P.
//
// One workgroup = 4 waves = 128 query rows (32 per wave, one wave per SIMD) x one range of keys (the key
// axis is split over workgroups so ~256 of them fill the chip; a combine pass adds the ranges).  Per
// block of 32 keys:
//   * the 32-key V tile (pre-split x2 rows of the in-projection output) arrives by LDS-DMA one block
//     ahead, the 128 x 32 score tile two blocks ahead;
//   * lane l of a wave takes query l%32 and the 8 consecutive keys 8h .. 8h+7 (h = l/32) of each
//     16-key step -- exactly the B operand of v_mfma_f32_32x32x16_bf16 -- so P never leaves registers;
//     block kb+1's P is formed while block kb's products run (software pipeline);
//   * O^T += V^T . P, V^T fragments read with ds_read_b64_tr_b16 from the k-major V image (BF16X3: the
//     three split products hi.lo + lo.hi + hi.hi; BF16: hi.hi only).
// Measured variants: two waves per SIMD (8 waves, d split in halves, P handed
// between partner waves through LDS) ran 2-4 % slower than this form; an ablation puts ~30 of its
// ~95 us (C4) in the fixed costs (row statistics, partial-output stores, the combine pass).
// BF16X6 (round 6, the "fwd6" policy): V is DMA'd as the in-projection's fp32 rows (the same 4 dp bytes per key
// as an x2 row, so the same LDS image size), its 32-column chunk halves XOR-swizzled by key-row bit 3, and the
// V^T fragments are read as 8 ds_read_b32 per lane and split into hi / mid / lo bf16 planes in registers; P is
// split three ways too, and each term is the six products mm, hl, lh, hm, mh, hh (fp32-accurate).
#include "u2gnn_common.h"
#include <cmath>

#include <type_traits>

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((address_space(3))) void lds_void;

constexpr int FA_BM = 128;   // query rows per workgroup (4 waves x 32)
constexpr int FA_BN = 32;    // keys per block
constexpr int FA_NT = 256;
constexpr int S_IMG = FA_BM * FA_BN * 4;   // bytes of one score tile

// V image (x2 rows of 4*dp bytes, k-major for the transpose reads): byte b of k-row r stored at
// b ^ kr_swz(r) -- the four k-rows of one ds_read_b64_tr_b16 land in four different 64-B bank quarters.
__device__ __forceinline__ int kr_swz(int krow) { return ((krow & 1) << 4) | ((krow & 2) << 6); }
// score image: 128-B rows (32 keys); 16-B chunk c of row r stored at c ^ ((r >> 1) & 7), so the 16 rows a
// 16-lane group of a ds_read_b128 touches hit 16 distinct bank slots.
__device__ __forceinline__ int s_swz(int r) { return (r >> 1) & 7; }

// One 16-B LDS-DMA per lane: global base (wave-uniform, SGPRs) + 32-bit lane offset -> LDS (wave-uniform
// piece base in M0, lane-linear inside it).
// Written as an asm statement on purpose: the compiler does not count it, so it neither inserts a
// vmcnt(0) in front of the fragment reads of the OTHER stage (it cannot tell the two stages apart
// through a DMA) nor orders anything after it; every wait on these is the counted wait_vm below.
// M0 is reserved (never allocated) and nothing else in these kernels reads it, so it is not clobbered.
__device__ __forceinline__ const char *uniform_ptr(const char *p) {
    const uint64_t v = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return reinterpret_cast<const char *>(((uint64_t)hi << 32) | lo);
}

// base and m0 are wave-uniform by construction; the readfirstlanes only tell the compiler so (the "s"
// operands need SGPRs whatever its divergence analysis concludes)
__device__ __forceinline__ void dma16(const char *base, int off, unsigned m0) {
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2" ::"s"(__builtin_amdgcn_readfirstlane(m0)),
                 "v"(off), "s"(uniform_ptr(base))
                 : "memory");
}

// LDS byte address of a shared object (a link-time constant)
__device__ __forceinline__ unsigned lds_addr(const void *p) { return (unsigned)(size_t)(const lds_void *)p; }

// fp32 V image (BF16X6): 16-B chunk c of key row r stored at c ^ (8 ((r >> 3) & 1)), i.e. rows 8..15 (mod 16)
// swap the two 128-B halves of every 256-B column group: the 8 ds_read_b32 of a fragment have lanes l < 32
// reading key row k and lanes l >= 32 row k + 8, which then fall in opposite 32-bank halves
__device__ __forceinline__ int kr_swz6(int krow) { return ((krow >> 3) & 1) << 7; }

template <int DP, int NPL, int NT = FA_NT>
__device__ __forceinline__ void issue_v(const char *vbase, int64_t ld_bytes, unsigned img, int tid, int w) {
    constexpr int RB = 4 * DP;                      // bytes per k-row (x2: hi + lo bf16; x6: fp32)
    constexpr int NI = FA_BN * RB / (16 * NT);     // DMA instructions per thread
    static_assert(NI * 16 * NT == FA_BN * RB, "V tile / threads");
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int b = (i * NT + tid) * 16;
        const int kr = b / RB, pb = b % RB;
        dma16(vbase, (int)(kr * ld_bytes) + (pb ^ (NPL == 3 ? kr_swz6(kr) : kr_swz(kr))), img + (i * NT + 64 * w) * 16);
    }
}

// the 128 x 32 score tile: 16 KB, 1 KB per wave-instruction
template <int NT = FA_NT>
__device__ __forceinline__ void issue_s(const char *sbase, int64_t lds_bytes, unsigned img, int tid, int w) {
#pragma unroll
    for (int i = 0; i < S_IMG / (16 * NT); ++i) {
        const int c = i * NT + tid;          // 16-B chunk of the image
        const int r = c >> 3, q = (c & 7) ^ s_swz(r);
        dma16(sbase, (int)(r * lds_bytes) + q * 16, img + (i * NT + 64 * w) * 16);
    }
}

template <int N_>
__device__ __forceinline__ void wait_vm() {
    static_assert(N_ >= 0 && N_ <= 63, "vmcnt range");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N_) : "memory");
}

// V^T fragment reads (A operand: row = d, k = key).  Lane (g = l/16, q = (l/4)%4, p = l%4) reads k-row
// kr = 16 ks + 8 (g>>1) + q, columns 32 t + 16 (g&1) + 4p .. +3 of the hi and lo halves.  kr_swz(kr)
// depends on q only (bits 4 and 7); bit 7 is also bit 0 of the tile index t, so
//   (128 t + x) ^ kr_swz = (x ^ (16 (q&1))) + 128 (t ^ (q>>1))
// and each lane keeps one base per parity of t -- every other term is a compile-time offset.
struct VBase {
    int a[2], b[2];   // hi / lo half byte offsets for even / odd t
};

template <int DP>
__device__ __forceinline__ VBase v_base(int lane) {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int row = ((g >> 1) * 8 + q) * (4 * DP);
    const int x = (g & 1) * 64 + (p >> 1) * 32 + (p & 1) * 8;   // < 128, bit 4 clear
    const int sq = (q >> 1) & 1;
    VBase B;
    B.a[0] = row + x + 16 * (q & 1) + 128 * sq;
    B.b[0] = row + x + 16 * (1 - (q & 1)) + 128 * sq;
    B.a[1] = B.a[0] - 256 * sq;
    B.b[1] = B.b[0] - 256 * sq;
    return B;
}

template <int DP>
__device__ __forceinline__ void v_frag(const char *img, const VBase &B, int dt, int ks, bf16x8 &hi, bf16x8 &lo) {
    const char *a = img + B.a[dt & 1] + 128 * dt + ks * 64 * DP;
    const char *b = img + B.b[dt & 1] + 128 * dt + ks * 64 * DP;
    const s16x4 h0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(a));
    const s16x4 h1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(a + 16 * DP));
    const s16x4 l0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(b));
    const s16x4 l1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(b + 16 * DP));
    const s16x4 vh[2] = {h0, h1}, vl[2] = {l0, l1};
    hi = __builtin_bit_cast(bf16x8, vh);
    lo = __builtin_bit_cast(bf16x8, vl);
}

// BF16X6: the V^T fragment of d tile dt, k step ks (lane: d = 32 dt + l % 32, keys 16 ks + 8 (l / 32) + e) from
// the fp32 image as 8 ds_read_b32, split into three bf16 planes.  base[dt & 1] = this lane's byte offset
// (v_base6); every other term is a compile-time offset
template <int DP>
__device__ __forceinline__ void v_base6(int lane, int (&base)[2]) {
    const int li = lane & 31, h = lane >> 5;
    // key row 16 ks + 8 h + e, chunk (8 dt + li / 4) ^ 8 h = 8 (dt ^ h) + li / 4
    base[0] = 8 * h * 4 * DP + 128 * h + 4 * li;
    base[1] = 8 * h * 4 * DP - 128 * h + 4 * li;
}

template <int DP>
__device__ __forceinline__ void v_frag6(const char *img, const int (&base)[2], int dt, int ks, bf16x8 &hi, bf16x8 &mid,
                                        bf16x8 &lo) {
    const char *a = img + base[dt & 1] + 128 * dt + ks * 64 * DP;
    float x[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] = *reinterpret_cast<const float *>(a + e * 4 * DP);
    unsigned h[4], m[4], l[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) split3(x[2 * i], x[2 * i + 1], h[i], m[i], l[i]);
    hi = __builtin_bit_cast(bf16x8, h);
    mid = __builtin_bit_cast(bf16x8, m);
    lo = __builtin_bit_cast(bf16x8, l);
}

__device__ __forceinline__ void split8_h(const float *x, float sc, bf16x8 &hi, bf16x8 &lo) {
    unsigned h[4], l[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) split2h(x[2 * i], x[2 * i + 1], sc, h[i], l[i]);
    hi = __builtin_bit_cast(bf16x8, h);
    lo = __builtin_bit_cast(bf16x8, l);
}

__device__ __forceinline__ void split8_3(const float *x, bf16x8 &hi, bf16x8 &mid, bf16x8 &lo) {
    unsigned h[4], m[4], l[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) split3(x[2 * i], x[2 * i + 1], h[i], m[i], l[i]);
    hi = __builtin_bit_cast(bf16x8, h);
    mid = __builtin_bit_cast(bf16x8, m);
    lo = __builtin_bit_cast(bf16x8, l);
}

__device__ __forceinline__ void split8(const float *x, bf16x8 &hi, bf16x8 &lo) {
    unsigned h[4], l[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) split2<true>(x[2 * i], x[2 * i + 1], h[i], l[i]);
    hi = __builtin_bit_cast(bf16x8, h);
    lo = __builtin_bit_cast(bf16x8, l);
}

struct SpvP {
    const float *S;        // scores [rows_pad][lds]
    int64_t lds;
    const float *rowpart;  // EPI_STORE_ROWSTAT partials: [rows_pad][ld_rowpart] (max, sum) pairs
    int64_t ld_rowpart;
    int32_t ngroups;
    const __bf16 *qkv2;    // x2 [rows_pad][ldq2]; BF16X6: the fp32 in-projection output [rows_pad][ldq2 floats]
    int64_t ldq2;
    int64_t ld_vbytes;     // bytes per row of qkv2
    float *Pd;             // signed image [rows_pad][ldp]
    int64_t ldp;
    float *Opart;          // [nsplit][rows_pad][dp]
    float *O;              // direct: O itself [rows_pad][ldo] (no combine pass)
    int64_t ldo;
    int32_t direct;
    int32_t n_valid, rows_pad, kb_valid, kb_per_split, nsplit, qblocks;
    float p;
    uint64_t seed;
    const uint64_t *epoch;
    float h3_sp, h3_inv;   // F16X3: the pre-scale of P (a power of two) and the inverse of P's and V's
};

// (m, l) <- the log-sum-exp merge with (m2, l2); -inf maxima (empty groups) contribute nothing
__device__ __forceinline__ void lse_merge(float &m, float &l, float m2, float l2) {
    const float n = fmaxf(m, m2);
    const float e1 = m == -INFINITY ? 0.f : __expf(m - n);
    const float e2 = m2 == -INFINITY ? 0.f : __expf(m2 - n);
    l = l * e1 + l2 * e2;
    m = n;
}

// (max, 1/sum) of one row from its ngroups (max, sum exp) partials: the row's two lanes (h = 0, 1) take
// alternate pairs of groups, 8 loads in flight per lane, and merge at the end -- the same order in every
// workgroup of the row block
__device__ __forceinline__ void row_stat(const SpvP &P, int query, int h, float &M, float &inv) {
    const float4 *pr = reinterpret_cast<const float4 *>(P.rowpart + 2 * (int64_t)query * P.ld_rowpart);
    const int n4 = P.ngroups / 2;
    float m = -INFINITY, l = 0.f;
    for (int j0 = h; j0 < n4; j0 += 16) {
        float4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int j = j0 + 2 * u;
            v[u] = j < n4 ? pr[j] : make_float4(-INFINITY, 0.f, -INFINITY, 0.f);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            lse_merge(m, l, v[u].x, v[u].y);
            lse_merge(m, l, v[u].z, v[u].w);
        }
    }
    const float m2 = __shfl_xor(m, 32, 64), l2 = __shfl_xor(l, 32, 64);
    if (h == 0) {
        lse_merge(m, l, m2, l2);
    } else {   // the same merge, operands in lane-0 order, so both lanes agree bit for bit
        float mm = m2, ll = l2;
        lse_merge(mm, ll, m, l);
        m = mm, l = ll;
    }
    M = m, inv = 1.f / l;
}

// this lane's P for keys kb*32 + 16 ks + 8 h .. +7 (ks = 0, 1: the B operands of the block's two 16-key
// steps), from the score tile simg; writes the signed image and returns the kept P/(1-p) split to bf16.
// No masks: keys >= n_valid hold -inf in S (EPI_STORE_ROWSTAT) and padded query rows have mb = +inf, so
// both reach exp2(-inf) = 0.
struct PRow {
    int r, h;
    float mb, inv, sc, hsc;   // hsc: F16X3 pre-scale of the kept probabilities
    uint32_t rkey, thr;
    float *prow;
};

template <int NPL>
__device__ __forceinline__ void p_half(const PRow &R, const char *simg, int kb, int ks, bf16x8 (&pp)[3]) {
    const int c = 4 * ks + 2 * R.h;   // logical 16-B chunk of the row
    const char *rowp = simg + R.r * 128;
    const float4 a = *reinterpret_cast<const float4 *>(rowp + ((c ^ s_swz(R.r)) << 4));
    const float4 b = *reinterpret_cast<const float4 *>(rowp + (((c + 1) ^ s_swz(R.r)) << 4));
    float sv[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    // pin the two vector reads (the compiler otherwise splits them into single-element reads)
#pragma unroll
    for (int t = 0; t < 8; ++t) asm("" : "+v"(sv[t]));
    const int kbase = kb * FA_BN + 16 * ks + 8 * R.h;   // even: keys kbase + 2q, + 2q + 1 share hash q
    uint32_t hs[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) hs[q] = u2gnn_pair_hash(R.rkey, (uint32_t)(kbase >> 1) + q);
    float pv[8], img[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        const float pr = __builtin_amdgcn_exp2f(sv[t] * 1.4426950408889634f - R.mb) * R.inv;
        const bool kp = (t & 1) ? u2gnn_keep_hi(hs[t >> 1], R.thr) : u2gnn_keep_lo(hs[t >> 1], R.thr);
        const float ps = pr * R.sc;
        pv[t] = kp ? ps : 0.f;
        img[t] = kp ? ps : -pr;
    }
    float *dst = R.prow + kbase;
#ifndef SPV_NO_STORE
    *reinterpret_cast<float4 *>(dst) = make_float4(img[0], img[1], img[2], img[3]);
    *reinterpret_cast<float4 *>(dst + 4) = make_float4(img[4], img[5], img[6], img[7]);
#else
    if (img[0] == 123.f) *dst = img[1] + img[2] + img[3] + img[4] + img[5] + img[6] + img[7];
#endif
    if constexpr (NPL == 3) split8_3(pv, pp[0], pp[1], pp[2]);
    else if constexpr (NPL == 4) split8_h(pv, R.hsc, pp[0], pp[1]);
    else split8(pv, pp[0], pp[1]);
}

template <int NPL>
__device__ __forceinline__ void p_block(const PRow &R, const char *simg, int kb, bf16x8 (&pp)[2][3]) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) p_half<NPL>(R, simg, kb, ks, pp[ks]);
}

// O^T += V^T . P over one block (V image vimg, P operands ph / pl); fragments of d tile t + 1 are read
// while the products of tile t run
template <int DP, int NPL>
__device__ __forceinline__ void pv_block(const char *vimg, const VBase &vb, const int (&vb6)[2], const bf16x8 (&pp)[2][3],
                                         f32x16 (&o)[DP / 32]) {
    constexpr int DT = DP / 32;
    if constexpr (NPL == 3) {
        // bf16x6: one d tile's fragments at a time (ks 1's reads and splits under ks 0's six products; a second
        // buffer for tile t + 1 spilled at dp = 384)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)   // (k step outermost: ks 0's P planes die before ks 1's tiles)
#pragma unroll
            for (int t = 0; t < DT; ++t) {   // smallest terms first: mm, hl, lh, hm, mh, then hh
                bf16x8 f[3];
                v_frag6<DP>(vimg, vb6, t, ks, f[0], f[1], f[2]);
                const bf16x8(&q)[3] = pp[ks];
                o[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f[1], q[1], o[t], 0, 0, 0);
                o[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f[0], q[2], o[t], 0, 0, 0);
                o[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f[2], q[0], o[t], 0, 0, 0);
                o[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f[0], q[1], o[t], 0, 0, 0);
                o[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f[1], q[0], o[t], 0, 0, 0);
                o[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f[0], q[0], o[t], 0, 0, 0);
            }
        return;
    }
    bf16x8 v[2][2][3];   // [buffer][ks][plane]
    auto frag = [&](int t, int ks, bf16x8 (&f)[3]) __attribute__((always_inline)) {
        v_frag<DP>(vimg, vb, t, ks, f[0], f[1]);
    };
    frag(0, 0, v[0][0]);
    frag(0, 1, v[0][1]);
#pragma unroll
    for (int t = 0; t < DT; ++t) {
        const int cur = t & 1;
        if (t + 1 < DT) {
            frag(t + 1, 0, v[cur ^ 1][0]);
            frag(t + 1, 1, v[cur ^ 1][1]);
        }
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const bf16x8(&f)[3] = v[cur][ks];
            const bf16x8(&q)[3] = pp[ks];
            if constexpr (NPL == 4) {   // f16x3: the x2 rows hold fp16 planes (U2GNN_H3_X2_EXP), P split likewise
                const auto h = [](bf16x8 v) { return __builtin_bit_cast(f16x8, v); };
                o[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(h(f[0]), h(q[1]), o[t], 0, 0, 0);
                o[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(h(f[1]), h(q[0]), o[t], 0, 0, 0);
                o[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(h(f[0]), h(q[0]), o[t], 0, 0, 0);
            } else {
                if constexpr (NPL >= 2) {
                    o[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f[0], q[1], o[t], 0, 0, 0);
                    o[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f[1], q[0], o[t], 0, 0, 0);
                }
                o[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f[0], q[0], o[t], 0, 0, 0);
            }
        }
    }
}

// Interleave hint for the scheduler: per matrix product, a few LDS reads and the VALU share of the next
// block's probabilities (~450 VALU per block: 6 per product in BF16X3, 18 in BF16), so the in-order wave
// issues them while the matrix pipe is busy (one wave per SIMD: nothing else would cover them).
template <int NMFMA, int NVALU>
__device__ __forceinline__ void interleave_hint() {
#pragma unroll
    for (int i = 0; i < NMFMA; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);       // MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);       // DS read
        __builtin_amdgcn_sched_group_barrier(0x002, NVALU, 0);   // VALU
    }
}

// Workgroup id -> (query block, key range): consecutive ids go to different XCDs (b and b + 8 share one),
// so deal the split-major list out in contiguous chunks per XCD -- the workgroups of one key range then
// share one L2 for their V tiles.
__device__ __forceinline__ void spv_block(int id, int total, int qblocks, int &qb, int &split) {
    const int x = id & 7, slot = id >> 3;
    const int base = total >> 3, extra = total & 7;
    const int pos = x * base + min(x, extra) + slot;
    split = pos / qblocks;
    qb = pos - split * qblocks;
}

// NPL: planes per operand -- 1 (bf16), 2 (bf16x3: x2 V rows), 3 (bf16x6: fp32 V rows), 4 (f16x3: x2 rows of fp16
// planes, U2GNN_H3_X2_EXP)
template <int DP, int NPL>
__global__ void __launch_bounds__(FA_NT, 1) attn_softmax_pv_kernel(SpvP P) {
    constexpr int DT = DP / 32;              // 32-wide d tiles of O
    constexpr int VIMG = FA_BN * 4 * DP;     // bytes of one V image
    __shared__ __attribute__((aligned(1024))) char vst0[VIMG];
    __shared__ __attribute__((aligned(1024))) char vst1[VIMG];
    __shared__ __attribute__((aligned(1024))) char sst0[S_IMG];
    __shared__ __attribute__((aligned(1024))) char sst1[S_IMG];
    const uint64_t seed = u2gnn_seed(P.seed, P.epoch);
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    int qb, split;
    spv_block(blockIdx.x, P.qblocks * P.nsplit, P.qblocks, qb, split);
    const int qrow0 = qb * FA_BM;
    PRow R;
    R.r = 32 * w + (lane & 31);              // this lane's row inside the block
    R.h = lane >> 5;
    const int query = qrow0 + R.r;
    const int kb0 = split * P.kb_per_split;
    const int kb1 = min(kb0 + P.kb_per_split, P.kb_valid);
    const int64_t ld_bytes = P.ld_vbytes, lds_bytes = P.lds * 4;
    // byte offset of V (column 2 dp): 2 dp x2 columns of 4 B (hi + lo), or 2 dp fp32 columns -- 8 DP either way
    const char *vcol = reinterpret_cast<const char *>(P.qkv2) + 8 * DP;
    const char *srow0 = reinterpret_cast<const char *>(P.S + (int64_t)qrow0 * P.lds);
    const bool qvalid = query < P.n_valid;
    float M = 0.f, inv = 0.f;
#ifndef SPV_NO_ROWSTAT
    if (qb * FA_BM < P.n_valid) row_stat(P, query, R.h, M, inv);
#else
    M = 0.f, inv = 1e-3f;
#endif
    // retire those loads before any LDS-DMA is in flight (every later wait below is a counted one)
    wait_vm<0>();
    R.mb = qvalid ? M * 1.4426950408889634f : INFINITY;   // padded rows: exp2(s - inf) = 0
    R.inv = qvalid ? inv : 0.f;
    R.thr = u2gnn_keep_thr(P.p);
    R.sc = P.p > 0.f ? 1.f / (1.f - P.p) : 1.f;
    R.hsc = P.h3_sp;
    R.rkey = u2gnn_row_key(seed, (uint32_t)query);
    R.prow = P.Pd + (int64_t)query * P.ldp;
    const VBase vb = v_base<DP>(lane);
    int vb6[2];
    v_base6<DP>(lane, vb6);

    f32x16 o[DT];
#pragma unroll
    for (int t = 0; t < DT; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) o[t][i] = 0.f;

    // Software pipeline over the key blocks: iteration kb multiplies block kb's P (computed one iteration
    // earlier) into V(kb) while it forms block kb+1's P from the score tile S(kb+1); LDS holds V(kb) and
    // S(kb+1) for the current iteration and receives V(kb+1) and S(kb+2) by DMA.  The stages are separate
    // LDS objects and the loop is unrolled by two, so every access names its stage at compile time.
    auto issue_vt = [&](int kb, unsigned img) __attribute__((always_inline)) {
        issue_v<DP, NPL>(vcol + (int64_t)kb * FA_BN * ld_bytes, ld_bytes, img, tid, w);
    };
    auto issue_st = [&](int kb, unsigned img) __attribute__((always_inline)) {
        issue_s(srow0 + (int64_t)kb * FA_BN * 4, lds_bytes, img, tid, w);
    };
    bf16x8 pp[2][3];   // [ks][plane]
    // an iteration that also forms the next block's P (kb + 1 < kb1)
    auto body = [&](auto stage, int kb) __attribute__((always_inline)) {
        constexpr int STG = decltype(stage)::value;
        // V(kb), S(kb+1) landed (this wave's pieces: only the 4 image stores issued after those DMAs
        // may still be in flight), then everyone's; every wave is also done with V(kb-1) and S(kb), whose
        // stages the next DMAs overwrite
        wait_vm<4>();
        __builtin_amdgcn_s_barrier();
#ifndef SPV_NO_DMA
        issue_vt(kb + 1, lds_addr(STG ? vst0 : vst1));
        if (kb + 2 < kb1) issue_st(kb + 2, lds_addr(STG ? sst1 : sst0));
#endif
        bf16x8 np[2][3];
#ifndef SPV_NO_P
        p_block<NPL>(R, STG ? sst0 : sst1, kb + 1, np);
#else
#pragma unroll
        for (int q = 0; q < 3; ++q) np[0][q] = pp[1][q], np[1][q] = pp[0][q];
#endif
#ifndef SPV_NO_MFMA
        pv_block<DP, NPL>(STG ? vst1 : vst0, vb, vb6, pp, o);
#endif
#ifndef SPV_NO_HINT
        if constexpr (NPL != 3) interleave_hint<(NPL == 1 ? 2 : 6) * DT, NPL == 1 ? 18 : NPL == 4 ? 8 : 6>();
#endif
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int q = 0; q < 3; ++q) pp[ks][q] = np[ks][q];
    };
    auto last = [&](auto stage) __attribute__((always_inline)) {
        constexpr int STG = decltype(stage)::value;
        wait_vm<4>();
        __builtin_amdgcn_s_barrier();
        pv_block<DP, NPL>(STG ? vst1 : vst0, vb, vb6, pp, o);
    };
    if (kb0 < kb1) {
        issue_vt(kb0, lds_addr(vst0));
        issue_st(kb0, lds_addr(sst0));
        if (kb0 + 1 < kb1) issue_st(kb0 + 1, lds_addr(sst1));
        wait_vm<0>();
        __builtin_amdgcn_s_barrier();
        p_block<NPL>(R, sst0, kb0, pp);
        int kb = kb0;
        for (; kb + 2 < kb1; kb += 2) {
            body(std::integral_constant<int, 0>(), kb);
            body(std::integral_constant<int, 1>(), kb + 1);
        }
        if (kb + 1 < kb1) {
            body(std::integral_constant<int, 0>(), kb);
            last(std::integral_constant<int, 1>());
        } else {
            last(std::integral_constant<int, 0>());
        }
    }
    // ---- partial O of this key range: O^T lane layout = query l%32, d = 32 t + 8 g + 4 h .. +3
    // (direct: one key range and one query block cover everything -- O itself, padded rows 0 via P = 0)
    float *orow = P.direct ? P.O + (int64_t)query * P.ldo : P.Opart + ((int64_t)split * P.rows_pad + query) * DP;
    if constexpr (NPL == 4) {   // undo the pre-scales (exact)
#pragma unroll
        for (int t = 0; t < DT; ++t) o[t] *= P.h3_inv;
    }
#ifndef SPV_NO_OSTORE
#pragma unroll
    for (int t = 0; t < DT; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g)
            *reinterpret_cast<float4 *>(orow + 32 * t + 8 * g + 4 * R.h) =
                make_float4(o[t][4 * g], o[t][4 * g + 1], o[t][4 * g + 2], o[t][4 * g + 3]);
#else
    float acc = 0.f;
#pragma unroll
    for (int t = 0; t < DT; ++t) acc += o[t][0] + o[t][5];
    if (acc == 123.f) *orow = acc;
#endif
    if (P.direct) {   // the image's key padding of this block's rows (the combine pass's job otherwise)
        const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int r = w; r < FA_BM; r += FA_NT / 64) {
            float *prow = P.Pd + (int64_t)(qrow0 + r) * P.ldp;
            for (int c = P.kb_valid * FA_BN + 4 * lane; c < P.rows_pad; c += 256)
                *reinterpret_cast<float4 *>(prow + c) = z;
        }
    }
}

// O[row] = sum over the key ranges (fixed order s = 0, 1, ...); rows >= n_valid zero.  One thread per
// float4 of O with every range's load in flight (8 at a time).  Then the parts of the signed image no
// fused block wrote -- keys from kb_valid*32 on, rows of query blocks past n_valid -- one wave per row.
__global__ void __launch_bounds__(256) attn_pv_combine_kernel(const float *Opart, int nsplit, int rows_pad,
                                                              int n_valid, int dp, float *O, int64_t ldo, float *Pd,
                                                              int64_t ldp, int key_end, int row_end) {
    const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    const int c4 = dp >> 2;
    if (gid < (int64_t)rows_pad * c4) {
        const int row = (int)(gid / c4), c = (int)(gid - (int64_t)row * c4) * 4;
        float4 acc = z;
        if (row < n_valid) {
            const float *p = Opart + (int64_t)row * dp + c;
            const int64_t stride = (int64_t)rows_pad * dp;
            for (int s0 = 0; s0 < nsplit; s0 += 8) {
                float4 v[8];
#pragma unroll
                for (int q = 0; q < 8; ++q)
                    if (s0 + q < nsplit) v[q] = *reinterpret_cast<const float4 *>(p + (s0 + q) * stride);
#pragma unroll
                for (int q = 0; q < 8; ++q)
                    if (s0 + q < nsplit) acc.x += v[q].x, acc.y += v[q].y, acc.z += v[q].z, acc.w += v[q].w;
            }
        }
        *reinterpret_cast<float4 *>(O + (int64_t)row * ldo + c) = acc;
    }
    const int64_t row = gid >> 6;
    const int lane = (int)(gid & 63);
    if (row < rows_pad) {
        float *prow = Pd + row * ldp;
        for (int c = (row < row_end ? key_end : 0) + lane * 4; c < rows_pad; c += 256)
            *reinterpret_cast<float4 *>(prow + c) = z;
    }
}

inline int spv_nsplit(int64_t n_valid) {
    const int64_t qb = (n_valid + FA_BM - 1) / FA_BM;
    const int64_t kb = (n_valid + FA_BN - 1) / FA_BN;
    int64_t s = 256 / (qb > 0 ? qb : 1);   // one workgroup per CU: ~256 of them in one round (C5: 128 or 64
                                           // workgroups instead ran 0.83 / 0.90 vs 0.81 ms per step)
    if (s > kb) s = kb;
    if (s < 1) s = 1;
    return (int)s;
}

template <int DP>
void launch_spv(const SpvP &P, int npl, hipStream_t st) {
    const dim3 grid((unsigned)(P.qblocks * P.nsplit));
    if (npl == 4)
        hipLaunchKernelGGL((attn_softmax_pv_kernel<DP, 4>), grid, dim3(FA_NT), 0, st, P);
    else if (npl == 3)
        hipLaunchKernelGGL((attn_softmax_pv_kernel<DP, 3>), grid, dim3(FA_NT), 0, st, P);
    else if (npl == 2)
        hipLaunchKernelGGL((attn_softmax_pv_kernel<DP, 2>), grid, dim3(FA_NT), 0, st, P);
    else
        hipLaunchKernelGGL((attn_softmax_pv_kernel<DP, 1>), grid, dim3(FA_NT), 0, st, P);
}

}  // namespace

extern "C" {

int64_t u2gnn_attn_softmax_pv_ws_floats(int64_t n_valid, int64_t rows_pad, int64_t dp) {
    if (n_valid < 1 || rows_pad < n_valid || dp < 64 || dp % 64) return -1;
    return (int64_t)spv_nsplit(n_valid) * rows_pad * dp;
}

int u2gnn_attn_softmax_pv(const float *S, int64_t lds, const float *rowpart, int64_t ld_rowpart, int64_t ngroups,
                          const void *qkv2, int64_t ldq2, int64_t dp, float *Pd, int64_t ldp, float *O, int64_t ldo,
                          float *ws, int64_t ws_floats, int64_t n_valid, int64_t rows_pad, float p, uint64_t seed,
                          int32_t precision, void *stream) {
    if (!S || !rowpart || !qkv2 || !Pd || !O || !ws || n_valid < 1 || rows_pad < n_valid || rows_pad % FA_BM ||
        !(p < 1.f) || p < 0.f ||
        (precision != U2GNN_PREC_BF16X3 && precision != U2GNN_PREC_BF16 && precision != U2GNN_PREC_BF16X6 &&
         precision != U2GNN_PREC_F16X3))
        return U2GNN_E_ARG;
    const bool x6 = precision == U2GNN_PREC_BF16X6;   // qkv2 = the fp32 in-projection output, ldq2 in floats
    if (dp < 64 || dp > 384 || dp % 64 || ldq2 < (x6 ? 3 : 6) * dp || (ldq2 & (x6 ? 3 : 7)) || lds < rows_pad || (lds & 3) ||
        ldp < rows_pad || (ldp & 3) || ldo < dp || (ldo & 3) || ngroups < 2 || (ngroups & 1) ||
        ld_rowpart < ngroups || (ld_rowpart & 1) || ngroups > INT32_MAX)
        return U2GNN_E_ARG;
    if (((uintptr_t)S & 15) || ((uintptr_t)qkv2 & 15) || ((uintptr_t)Pd & 15) || ((uintptr_t)O & 15) ||
        ((uintptr_t)rowpart & 15) || ((uintptr_t)ws & 15))
        return U2GNN_E_ALIGN;
    // 32-bit byte offsets inside one block's DMA sources
    const int64_t ld_vbytes = ldq2 * (x6 ? 4 : 2);
    if ((int64_t)FA_BM * lds * 4 >= INT32_MAX || (int64_t)FA_BN * ld_vbytes >= INT32_MAX) return U2GNN_E_SHAPE;
    const int64_t need = u2gnn_attn_softmax_pv_ws_floats(n_valid, rows_pad, dp);
    if (need < 0 || ws_floats < need) return U2GNN_E_ARG;
    SpvP P;
    P.S = S;
    P.lds = lds;
    P.rowpart = rowpart;
    P.ld_rowpart = ld_rowpart;
    P.ngroups = (int32_t)ngroups;
    P.qkv2 = static_cast<const __bf16 *>(qkv2);
    P.ldq2 = ldq2;
    P.ld_vbytes = ld_vbytes;
    P.Pd = Pd;
    P.ldp = ldp;
    P.Opart = ws;
    P.O = O;
    P.ldo = ldo;
    P.nsplit = spv_nsplit(n_valid);
    P.qblocks = (int32_t)((n_valid + FA_BM - 1) / FA_BM);   // blocks of padding rows only: zeroed below
    P.n_valid = (int32_t)n_valid;
    P.rows_pad = (int32_t)rows_pad;
    P.kb_valid = (int32_t)((n_valid + FA_BN - 1) / FA_BN);
    // at most 4 key blocks and one query block over every padded row (C2's IMDBBINARY batches, ~80 nodes):
    // one workgroup walks all the keys and writes O and the image padding itself -- no combine launch (the
    // split saved less than the combine's launch; the O sums then run in key order in one accumulator)
    P.direct = P.kb_valid <= 4 && (int64_t)P.qblocks * FA_BM == rows_pad;
    if (P.direct) P.nsplit = 1;
    P.kb_per_split = (P.kb_valid + P.nsplit - 1) / P.nsplit;
    P.p = p;
    P.seed = seed;
    P.epoch = u2gnn_cur_epoch();
    // f16x3: V arrives pre-scaled by 2^U2GNN_H3_X2_EXP in its fp16 x2 rows; the kept probabilities (at most
    // 1/(1-p)) are scaled by 2^(15 - ceil(log2(1/(1-p)))) before their split (encoder_layer.cpp h3_prob_exp)
    int ep = 15;
    for (float m = p > 0.f ? 1.f / (1.f - p) : 1.f; m > 1.f; m *= 0.5f) --ep;
    P.h3_sp = std::ldexp(1.f, ep);
    P.h3_inv = std::ldexp(1.f, -(ep + U2GNN_H3_X2_EXP));
    hipStream_t st = u2gnn_stream(stream);
    const int npl = precision == U2GNN_PREC_F16X3 ? 4 : x6 ? 3 : precision == U2GNN_PREC_BF16X3 ? 2 : 1;
    switch (dp) {
#ifndef SPV_ONLY384   // (kernel experiments: build the dp = 384 instances only)
        case 64: launch_spv<64>(P, npl, st); break;
        case 128: launch_spv<128>(P, npl, st); break;
        case 192: launch_spv<192>(P, npl, st); break;
        case 256: launch_spv<256>(P, npl, st); break;
        case 320: launch_spv<320>(P, npl, st); break;
#endif
        default: launch_spv<384>(P, npl, st); break;
    }
    const int rc = u2gnn_launch_status();
    if (rc != U2GNN_OK || P.direct) return rc;
    const int64_t cthreads = rows_pad * (dp / 4) > rows_pad * 64 ? rows_pad * (dp / 4) : rows_pad * 64;
    hipLaunchKernelGGL(attn_pv_combine_kernel, dim3((unsigned)((cthreads + 255) / 256)), dim3(256), 0, st, ws, P.nsplit,
                       (int)rows_pad, (int)n_valid, (int)dp, O, ldo, Pd, ldp, P.kb_valid * FA_BN, P.qblocks * FA_BM);
    return u2gnn_launch_status();
}

}  // extern "C"
