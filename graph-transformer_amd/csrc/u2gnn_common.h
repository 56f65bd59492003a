// Shared device helpers for the U2GNN gfx950 kernels (wave64 reductions, dropout hash).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "u2gnn_hip.h"

#define U2GNN_WAVE 64

static inline int u2gnn_launch_status() {
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? U2GNN_OK : (int)e;
}

static inline hipStream_t u2gnn_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

// ---------------------------------------------------------------------------------------
// Dropout: counter-based keep decision.  keep(seed, i, j) = U(seed, i, j) >= p with U a 16-bit
// uniform: half of a murmur3 32-bit finaliser of (rowkey(seed, i) + (j / 2) * golden), the low half
// for even j, the high half for odd j -- one finaliser per two columns.  rowkey folds both seed
// halves and the row through the same finaliser.  32-bit integer work only, and the comparison in
// integers (U >= ceil(65536 p), exact for every p in [0, 1)): the N^2 attention dropout is the
// largest consumer.  The same (seed, i, j) regenerates the mask in backward; nothing is stored.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t u2gnn_fmix32(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    return h ^ (h >> 16);
}

__device__ __forceinline__ uint32_t u2gnn_row_key(uint64_t seed, uint32_t i) {
    return u2gnn_fmix32((uint32_t)seed ^ u2gnn_fmix32((uint32_t)(seed >> 32) ^ u2gnn_fmix32(i + 0x9E3779B9u)));
}

// Graph replay (ABI v6): every kernel that draws dropout decisions receives, beside its by-value
// seed, the launching device's seed-epoch pointer as it was at launch (u2gnn_set_seed_epoch; NULL = off;
// per device since ABI v17) and mixes the device-resident epoch into the seed, so a captured HIP graph
// draws new masks on every replay (u2gnn_step_advance bumps the epoch inside the graph).  Epoch 0 leaves
// the seed unchanged.
const uint64_t *u2gnn_cur_epoch();   // the current device's epoch pointer (head_ops.hip)
__device__ __forceinline__ uint64_t u2gnn_seed(uint64_t seed, const uint64_t *epoch) {
    return epoch ? seed ^ (*epoch * 0x9E3779B97F4A7C15ull) : seed;
}

// the integer threshold of keep probability 1 - p: U >= thr  <=>  U / 65536 >= p
__device__ __forceinline__ uint32_t u2gnn_keep_thr(float p) { return (uint32_t)ceilf(p * 65536.f); }

// the finaliser word of columns 2c, 2c + 1 of the row with key rkey
__device__ __forceinline__ uint32_t u2gnn_pair_hash(uint32_t rkey, uint32_t c) {
    return u2gnn_fmix32(rkey + c * 0x9E3779B9u);
}

// keep bits of columns 2c (low half of h) and 2c + 1 (high half)
__device__ __forceinline__ bool u2gnn_keep_lo(uint32_t h, uint32_t thr) { return (h & 0xFFFFu) >= thr; }
__device__ __forceinline__ bool u2gnn_keep_hi(uint32_t h, uint32_t thr) { return (h >> 16) >= thr; }

__device__ __forceinline__ bool u2gnn_keep_rk(uint32_t rkey, uint32_t j, uint32_t thr) {
    const uint32_t h = u2gnn_pair_hash(rkey, j >> 1);
    return (j & 1) ? u2gnn_keep_hi(h, thr) : u2gnn_keep_lo(h, thr);
}

__device__ __forceinline__ bool u2gnn_keep(uint64_t seed, uint32_t i, uint32_t j, float p) {
    return u2gnn_keep_rk(u2gnn_row_key(seed, i), j, u2gnn_keep_thr(p));
}

// ---------------------------------------------------------------------------------------
// wave64 reductions (DPP/permute lowered by the compiler from __shfl_xor)
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// padded -> real block map used by pack / unpack kernels
__device__ __forceinline__ int64_t blk_map(int64_t i, int64_t blk_pad, int64_t blk_real, bool *valid) {
    const int64_t b = i / blk_pad, r = i - b * blk_pad;
    *valid = r < blk_real;
    return b * blk_real + r;
}

// ---------------------------------------------------------------------------------------
// x2 format (pre-split fp32, include/u2gnn_hip.h): bf16 hi/lo pairs, hi = bf16_rne(x), lo = bf16_rne(x - hi)
// ---------------------------------------------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

typedef float f32x2 __attribute__((ext_vector_type(2)));

// (x0, x1) -> packed bf16 hi pair and, for SPLIT, the packed bf16 residual pair:
// one v_cvt_pk_bf16_f32, two bit ops, one packed subtraction (v_pk_add_f32: both residuals, exact), one more
// cvt_pk (5 VALU per pair; two scalar subtractions made it 6, the same bits).
template <bool SPLIT>
__device__ __forceinline__ void split2(float x0, float x1, unsigned &h, unsigned &l) {
    // opaque to the optimizer: otherwise it re-derives bf16(x0) with a second cvt instead of
    // shifting the packed pair
#ifdef U2GNN_EXP_NOSPLIT
    h = __float_as_uint(x0) ^ __float_as_uint(x1); l = h; return;
#endif
    asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(h) : "v"(x0), "v"(x1));
    if constexpr (SPLIT) {
        const f32x2 r = f32x2{x0, x1} - f32x2{__uint_as_float(h << 16), __uint_as_float(h & 0xffff0000u)};
        l = __builtin_bit_cast(unsigned, bf16x2{(__bf16)r.x, (__bf16)r.y});
    }
}

// (x0, x1) -> packed bf16 pairs hi, mid, lo with x = hi + mid + lo: hi = bf16(x), mid = bf16(x - hi),
// lo = bf16(x - hi - mid); both residuals are exact in fp32, so the three planes carry every bit of x
// (U2GNN_PREC_BF16X6).  3 cvt_pk + 4 bit ops + 4 subtractions per pair.
__device__ __forceinline__ void split3(float x0, float x1, unsigned &h, unsigned &m, unsigned &l) {
    asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(h) : "v"(x0), "v"(x1));
    const float r0 = x0 - __uint_as_float(h << 16), r1 = x1 - __uint_as_float(h & 0xffff0000u);
    asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(m) : "v"(r0), "v"(r1));
    const float s0 = r0 - __uint_as_float(m << 16), s1 = r1 - __uint_as_float(m & 0xffff0000u);
    asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(l) : "v"(s0), "v"(s1));
}

// (x0, x1) -> packed fp16 pairs hi, lo with hi = fp16_rne(x), lo = fp16_rne(x - hi) (U2GNN_PREC_F16X3): the
// residual is exact in fp32, so the pair carries 22 significant bits of x (fewer where lo is subnormal)
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
// ... of the pre-scaled pair (s x0, s x1), s a power of two: hi = fp16_rne(s x) and lo = fp16_rne(s x - hi), each one
// mixed-precision fma (v_fma_mix{lo,hi}_f16: the product and the difference exact, one rounding), 4 VALU per pair --
// the compiler's form of the same arithmetic formed hi twice (mix + mul + cvt_pk) and took 7, the same bits
__device__ __forceinline__ void split2h(float x0, float x1, float s, unsigned &h, unsigned &l) {
    asm("v_fma_mixlo_f16 %0, %1, %2, 0\n\t"
        "v_fma_mixhi_f16 %0, %1, %3, 0"
        : "=&v"(h) : "v"(s), "v"(x0), "v"(x1));
    asm("v_fma_mixlo_f16 %0, %1, %2, -%4 op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixhi_f16 %0, %1, %3, -%4 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
        : "=&v"(l) : "v"(s), "v"(x0), "v"(x1), "v"(h));
}

// x2 store of four consecutive columns in the f16x3 form: fp16 hi / lo of sc * o (the same layout)
__device__ __forceinline__ void store_x2h_4(__bf16 *Cx2, int64_t ldcx2, int row, int col, float4 o, float sc) {
    unsigned h0, h1, l0, l1;
    split2h(o.x, o.y, sc, h0, l0);
    split2h(o.z, o.w, sc, h1, l1);
    __bf16 *b = Cx2 + (int64_t)row * ldcx2 + 2 * (col & ~7) + (col & 7);
    *reinterpret_cast<uint2 *>(b) = make_uint2(h0, h1);
    *reinterpret_cast<uint2 *>(b + 8) = make_uint2(l0, l1);
}

// x2 store of four consecutive columns (col % 4 == 0): hi at 16*(col/8) + col%8, lo 8 further
__device__ __forceinline__ void store_x2_4(__bf16 *Cx2, int64_t ldcx2, int row, int col, float4 o) {
    unsigned h0, h1, l0, l1;
    split2<true>(o.x, o.y, h0, l0);
    split2<true>(o.z, o.w, h1, l1);
    __bf16 *b = Cx2 + (int64_t)row * ldcx2 + 2 * (col & ~7) + (col & 7);
    *reinterpret_cast<uint2 *>(b) = make_uint2(h0, h1);
    *reinterpret_cast<uint2 *>(b + 8) = make_uint2(l0, l1);
}

