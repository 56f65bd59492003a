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
// Dropout: counter-based keep decision.  keep(seed, i, j) = U(seed, i, j) >= p with U a
// 24-bit uniform from a splitmix64 finaliser of (seed + (i<<32|j) * golden).  The same
// (seed, i, j) regenerates the mask in backward, so masks are never stored.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t u2gnn_mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

__device__ __forceinline__ bool u2gnn_keep(uint64_t seed, uint32_t i, uint32_t j, float p) {
    const uint64_t x = seed + ((((uint64_t)i) << 32) | (uint64_t)j) * 0x9E3779B97F4A7C15ULL;
    const uint32_t u = (uint32_t)(u2gnn_mix64(x) >> 40);  // 24 bits
    return (float)u * (1.0f / 16777216.0f) >= p;
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
