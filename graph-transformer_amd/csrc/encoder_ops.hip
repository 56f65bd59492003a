// Row-wise and bandwidth-bound kernels of the U2GNN encoder on gfx950:
// neighbour gather, attention softmax+dropout, post-LN forward/backward, split-K reduce /
// parameter pack, bias-gradient column sums.  All are HBM-bound streaming passes:
// one wave64 per row, coalesced lane-contiguous accesses, fp32 throughout.
#include "u2gnn_common.h"

#include <algorithm>
#include <cstring>
#include <vector>

namespace {

// ------------------------------------------------------------------------------------------
// a2 neighbour gather (pytorch_U2GNN_Sup.py:32,39): one wave per destination row, every source
// load of the row issued before its stores (restrict pointers, unrolled).  MODE 1: 16-byte
// source rows and destination rows, a float4 of columns per lane in each 256-column chunk.
// MODE 2: 4-byte-aligned source rows (X_concat with d = 367 starts rows at arbitrary 4-byte
// offsets): lane-consecutive 4-byte loads and stores, 16 columns per lane in flight.  Both need
// d_pad <= 1024.  MODE 0: the plain per-column loop for anything else.
// ------------------------------------------------------------------------------------------
template <int MODE>
__global__ void __launch_bounds__(256) gather_rows_kernel(const float *__restrict__ src, int64_t ld_src,
                                                          int64_t src_rows, const int64_t *__restrict__ idx,
                                                          int64_t idx_stride, float *__restrict__ dst,
                                                          int64_t ld_dst, int64_t n_rows, int64_t n_rows_pad,
                                                          int64_t d, int64_t d_pad, int32_t *err) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= n_rows_pad) return;
    float *o = dst + row * ld_dst;
    int64_t s = -1;
    if (row < n_rows) {
        s = idx[row * idx_stride];
        if (s < 0 || s >= src_rows) {
            if (lane == 0 && err) atomicExch(err, 1);
            s = -1;
        }
    }
    const float *in = src + (s < 0 ? 0 : s) * ld_src;
    if constexpr (MODE == 1) {
        float4 v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int c = 256 * j + 4 * lane;
            v[j] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (s < 0 || c >= d) continue;
            if (c + 3 < d) {
                v[j] = *reinterpret_cast<const float4 *>(in + c);
            } else {
                v[j].x = in[c];
                if (c + 1 < d) v[j].y = in[c + 1];
                if (c + 2 < d) v[j].z = in[c + 2];
            }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int c = 256 * j + 4 * lane;
            if (c < d_pad) *reinterpret_cast<float4 *>(o + c) = v[j];
        }
    } else if constexpr (MODE == 2) {
        float v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int c = 64 * j + lane;
            v[j] = (s >= 0 && c < d) ? in[c] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int c = 64 * j + lane;
            if (c < d_pad) o[c] = v[j];
        }
    } else {
        for (int64_t c = lane; c < d_pad; c += 64) o[c] = (s >= 0 && c < d) ? in[c] : 0.f;
    }
}

// a2 gather for 4-byte-aligned source rows, d_pad <= 512 (X_concat, d = 367): GR_RPW rows per wave
// (their index loads, then all their source loads in flight), XCD-aware block order and, for WIDE,
// 16-byte stores -- each wave transposes its rows through a private LDS image (lane-consecutive
// 4-byte ds_write, ds_read_b128 of 4 consecutive columns per lane; both conflict-free), so a row
// leaves as 16-byte pieces instead of 6 x 256-B dword stores.  ld_dst % 4 == 0 and dst 16-byte
// aligned (checked by the caller); WIDE also needs d_pad % 4 == 0.
// Measured on one C4 batch (68374 x 367 -> [68608, 384], tools/gather_ab.py, profiles/r02/gather_ab.txt):
// one wave per row (MODE 2) 29.4 us; 2 rows/wave 24.7; + XCD order 21.6; + wide stores 18.6;
// 1 row/wave + XCD + wide 17.8 us (= 6.3 TB/s algorithmic; a 105 MB fill_ takes 14.8 us).  Wide stores
// alone, without the XCD order, lose (27.1 vs 26.2 us at 4 rows/wave); non-temporal stores lose too.
template <int GR_RPW, bool WIDE, bool XCD>
__global__ void __launch_bounds__(256) gather_rows_multi_kernel(const float *__restrict__ src, int64_t ld_src,
                                                                int64_t src_rows, const int64_t *__restrict__ idx,
                                                                int64_t idx_stride, float *__restrict__ dst,
                                                                int64_t ld_dst, int64_t n_rows, int64_t n_rows_pad,
                                                                int64_t d, int64_t d_pad, int32_t *err) {
    __shared__ __attribute__((aligned(16))) float img[4][WIDE ? GR_RPW : 1][WIDE ? 512 : 4];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // XCD: blocks are dealt round-robin to the 8 XCDs; remap so XCD x walks one contiguous eighth of
    // the rows (gridDim.x % 8 == 0) -- a graph's neighbour rows then stay in one XCD's L2
    const int64_t blk = XCD ? (int64_t)(blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3) : blockIdx.x;
    const int64_t row0 = (blk * 4 + w) * GR_RPW;
    if (row0 >= n_rows_pad) return;
    int64_t s[GR_RPW];
#pragma unroll
    for (int i = 0; i < GR_RPW; ++i) {
        const int64_t row = row0 + i;
        s[i] = -1;
        if (row < n_rows) {
            const int64_t t = idx[row * idx_stride];
            if (t < 0 || t >= src_rows) {
                if (lane == 0 && err) atomicExch(err, 1);
            } else {
                s[i] = t;
            }
        }
    }
    float v[GR_RPW][8];
#pragma unroll
    for (int i = 0; i < GR_RPW; ++i) {
        const float *in = src + (s[i] < 0 ? 0 : s[i]) * ld_src;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int c = 64 * j + lane;
            v[i][j] = (s[i] >= 0 && c < d) ? in[c] : 0.f;
        }
    }
    if constexpr (WIDE) {
#pragma unroll
        for (int i = 0; i < GR_RPW; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j) img[w][i][64 * j + lane] = v[i][j];
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int i = 0; i < GR_RPW; ++i) {
            const int64_t row = row0 + i;
            if (row >= n_rows_pad) break;
            float *o = dst + row * ld_dst;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int c = 256 * j + 4 * lane;
                if (c < d_pad) *reinterpret_cast<float4 *>(o + c) = *reinterpret_cast<const float4 *>(&img[w][i][c]);
            }
        }
    } else {
#pragma unroll
        for (int i = 0; i < GR_RPW; ++i) {
            const int64_t row = row0 + i;
            if (row >= n_rows_pad) break;
            float *o = dst + row * ld_dst;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int c = 64 * j + lane;
                if (c < d_pad) o[c] = v[i][j];
            }
        }
    }
}

// an index outside [0, dst_rows) adds nothing and sets *err (F.embedding raises IndexError there)
__global__ void __launch_bounds__(256) scatter_add_rows_kernel(const float *src, int64_t ld_src, const int64_t *idx,
                                                               int64_t idx_stride, float *dst, int64_t ld_dst,
                                                               int64_t dst_rows, int64_t n_rows, int64_t d,
                                                               int32_t *err) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= n_rows) return;
    const int64_t t = idx[row * idx_stride];
    if (t < 0 || t >= dst_rows) {
        if (lane == 0 && err) atomicExch(err, 1);
        return;
    }
    for (int64_t c = lane; c < d; c += 64) atomicAdd(dst + t * ld_dst + c, src[row * ld_src + c]);
}

// ------------------------------------------------------------------------------------------
// split-K slab reduce + padded->real unpack; pack real->padded
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ float4 ld4(const float *p) { return *reinterpret_cast<const float4 *>(p); }
__device__ __forceinline__ float4 add4(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }

// One wave per padded row, a float4 of columns per lane; the slab loop keeps 4 independent
// 16-byte loads in flight.  Rows/columns outside the real blocks are skipped; the real
// destination is written with 16-byte stores when the column map is the identity and aligned.
// sum of n_slab float4 slices at p, p + slab_stride, ... in the fixed order of every slab reduction:
// a += s0, s4, ...; b += s1, s5, ...; e += s2, ...; f += s3, ...; then (a + b) + (e + f); 8 loads in flight
__device__ __forceinline__ float4 slab_sum4(const float *p, int n_slab, int64_t slab_stride) {
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a, e = a, f = a;
    int z = 0;
    for (; z + 8 <= n_slab; z += 8) {
        float4 l[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) l[q] = ld4(p + (int64_t)(z + q) * slab_stride);
        a = add4(a, l[0]), b = add4(b, l[1]), e = add4(e, l[2]), f = add4(f, l[3]);
        a = add4(a, l[4]), b = add4(b, l[5]), e = add4(e, l[6]), f = add4(f, l[7]);
    }
    if (z + 4 <= n_slab) {
        float4 l[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) l[q] = ld4(p + (int64_t)(z + q) * slab_stride);
        a = add4(a, l[0]), b = add4(b, l[1]), e = add4(e, l[2]), f = add4(f, l[3]);
        z += 4;
    }
    if (z < n_slab) {   // the last 1-3 slices: loaded together from clamped addresses, then added in order (a loop
        // here waited out one memory round trip per slice, tools/isa_waits.py)
        const int z1 = min(z + 1, n_slab - 1), z2 = min(z + 2, n_slab - 1);
        const float4 l0 = ld4(p + (int64_t)z * slab_stride), l1 = ld4(p + (int64_t)z1 * slab_stride);
        const float4 l2 = ld4(p + (int64_t)z2 * slab_stride);
        a = add4(a, l0);
        if (z + 1 < n_slab) a = add4(a, l1);
        if (z + 2 < n_slab) a = add4(a, l2);
    }
    return add4(add4(a, b), add4(e, f));
}

// The bodies of the reduction kernels take their block coordinates as arguments, so that the batched
// launch (reduce_batch_kernel, u2gnn_reduce_batch) runs the very same per-element arithmetic.
__device__ __forceinline__ void slab_reduce_body(const float *src, int n_slab, int64_t slab_stride, int64_t rows_pad,
                                                 int64_t cols_pad, int64_t ld_src, int64_t rbp, int64_t rbr,
                                                 int64_t cbp, int64_t cbr, float *dst, int64_t ld_dst, float alpha,
                                                 int accumulate, int vec_store, int64_t i) {
    // one float4 of the output per thread (weight-gradient outputs have only d or ff rows: a wave per
    // row left the chip latency-bound); 8 slab loads in flight, summed in the fixed order
    // a += s0, s4, ...; b += s1, s5, ...; e += s2, ...; f += s3, ...; then (a + b) + (e + f)
    const int64_t c4 = cols_pad >> 2;
    if (i >= rows_pad * c4) return;
    const int64_t r = i / c4, c = (i - r * c4) * 4;
    bool vr;
    const int64_t rr = blk_map(r, rbp, rbr, &vr);
    if (!vr) return;
    const float4 t = slab_sum4(src + r * ld_src + c, n_slab, slab_stride);
    if (vec_store) {
        float *o = dst + rr * ld_dst + c;
        float4 v = make_float4(alpha * t.x, alpha * t.y, alpha * t.z, alpha * t.w);
        if (accumulate) v = add4(v, ld4(o));
        *reinterpret_cast<float4 *>(o) = v;
    } else {
        const float x[4] = {t.x, t.y, t.z, t.w};
        float *orow = dst + rr * ld_dst;
        int64_t cc[4];
        bool vc[4];
        float ov[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int q = 0; q < 4; ++q) cc[q] = blk_map(c + q, cbp, cbr, &vc[q]);
        // the four old values loaded before any store (blk_map is injective: no aliasing; clamped addresses): a
        // load -> store per column waited out four dependent memory round trips
        if (accumulate)
#pragma unroll
            for (int q = 0; q < 4; ++q) ov[q] = orow[vc[q] ? cc[q] : 0];
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (vc[q]) orow[cc[q]] = accumulate ? ov[q] + alpha * x[q] : alpha * x[q];
    }
}

__global__ void __launch_bounds__(256) slab_reduce_kernel(const float *src, int n_slab, int64_t slab_stride,
                                                          int64_t rows_pad, int64_t cols_pad, int64_t ld_src,
                                                          int64_t rbp, int64_t rbr, int64_t cbp, int64_t cbr,
                                                          float *dst, int64_t ld_dst, float alpha, int accumulate,
                                                          int vec_store) {
    slab_reduce_body(src, n_slab, slab_stride, rows_pad, cols_pad, ld_src, rbp, rbr, cbp, cbr, dst, ld_dst, alpha,
                     accumulate, vec_store, (int64_t)blockIdx.x * 256 + threadIdx.x);
}

__global__ void __launch_bounds__(256) pack_padded_kernel(const float *src, int64_t ld_src, int64_t rows_pad,
                                                          int64_t cols_pad, int64_t rbp, int64_t rbr, int64_t cbp,
                                                          int64_t cbr, float *dst, int64_t ld_dst) {
    const int64_t total = rows_pad * cols_pad;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        const int64_t r = i / cols_pad, c = i - r * cols_pad;
        bool vr, vc;
        const int64_t rr = blk_map(r, rbp, rbr, &vr);
        const int64_t cc = blk_map(c, cbp, cbr, &vc);
        dst[r * ld_dst + c] = (vr && vc) ? src[rr * ld_src + cc] : 0.f;
    }
}

// many pack jobs in one launch: the descriptors travel by value in the kernel arguments
constexpr int PACK_MAX = 32;
struct PackBatch {
    u2gnn_pack_desc d[PACK_MAX];
    uint64_t *adv_epoch;   // u2gnn_pack_padded_multi_adv: the step state bumped by block (0, 0)
    int64_t *adv_t;
};

// the graph-replay step advance (u2gnn_step_advance) carried by the step's first launch, the weight pack
__device__ __forceinline__ void pack_advance(const PackBatch &pb) {
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
        if (pb.adv_epoch) *pb.adv_epoch += 1;
        if (pb.adv_t) *pb.adv_t += 1;
    }
}

// Many padded-copy jobs in one launch: blockIdx.y = job, blockIdx.x = a group of PACK_RB rows, each
// thread one column per 256 (the column map computed once per column, the row map once per row, in
// 32-bit arithmetic: the first version's two 64-bit divisions per element held the C4 launch at 26 us
// for 42 MB).  Jobs whose extents do not fit 32 bits use pack_multi64_kernel.
constexpr uint32_t PACK_RB = 8;

__global__ void __launch_bounds__(256) pack_multi_kernel(PackBatch pb) {
    pack_advance(pb);
    const u2gnn_pack_desc &D = pb.d[blockIdx.y];
    const uint32_t rows = (uint32_t)D.rows_pad, cols = (uint32_t)D.cols_pad;
    const uint32_t r0 = blockIdx.x * PACK_RB;
    if (r0 >= rows) return;
    const uint32_t rbp = (uint32_t)D.rblk_pad, rbr = (uint32_t)D.rblk_real;
    const uint32_t cbp = (uint32_t)D.cblk_pad, cbr = (uint32_t)D.cblk_real;
    const uint32_t nr = min(PACK_RB, rows - r0);
    for (uint32_t c = threadIdx.x; c < cols; c += 256) {
        const uint32_t cb = c / cbp, ci = c - cb * cbp;
        const bool vc = ci < cbr;
        const uint32_t cc = cb * cbr + ci;
        float v[PACK_RB];
#pragma unroll
        for (uint32_t k = 0; k < PACK_RB; ++k) {   // every row's load in flight before the stores
            const uint32_t r = r0 + k, rb = r / rbp, ri = r - rb * rbp;
            v[k] = (k < nr && vc && ri < rbr) ? D.src[(int64_t)(rb * rbr + ri) * D.ld_src + cc] : 0.f;
        }
#pragma unroll
        for (uint32_t k = 0; k < PACK_RB; ++k)
            if (k < nr) D.dst[(int64_t)(r0 + k) * D.ld_dst + c] = v[k];
    }
}

__global__ void __launch_bounds__(256) pack_multi64_kernel(PackBatch pb) {
    pack_advance(pb);
    const u2gnn_pack_desc &D = pb.d[blockIdx.y];
    const int64_t total = D.rows_pad * D.cols_pad;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        const int64_t r = i / D.cols_pad, c = i - r * D.cols_pad;
        bool vr, vc;
        const int64_t rr = blk_map(r, D.rblk_pad, D.rblk_real, &vr);
        const int64_t cc = blk_map(c, D.cblk_pad, D.cblk_real, &vc);
        D.dst[r * D.ld_dst + c] = (vr && vc) ? D.src[rr * D.ld_src + cc] : 0.f;
    }
}

// column sums, stage 1: block = CS_ROWS rows x 256 columns; each lane owns a float4 of columns,
// each wave CS_ROWS/4 rows (all its loads in flight at once), ws[chunk][col] via LDS.  Small row
// chunks give ~Np/16 x cols/256 blocks, enough waves to cover HBM latency; token-sized inputs
// (neighbour mode) fold rep groups into one chunk so that at most COLSUM_MAX_CHUNKS partial rows
// reach the column-parallel stage 2 (rep = 1 below 8K rows: C4 sums are unchanged).
constexpr int CS_ROWS = 16;
constexpr int64_t COLSUM_MAX_CHUNKS = 512;

template <bool FOLD>
__device__ __forceinline__ void colsum_partial_body(const float *X, int64_t rows, int64_t cols_pad, int64_t ld, int rep,
                                                    float *ws, int bx, int by) {
    __shared__ float4 red[4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t c = ((int64_t)bx * 64 + lane) * 4;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    const int nrep = FOLD ? rep : 1;     // compile-time 1 unless folding: the C4 body stays straight-line
    for (int it = 0; it < nrep; ++it) {  // a chunk = rep consecutive CS_ROWS-row groups
        const int64_t r0 = ((int64_t)by * nrep + it) * CS_ROWS + w * (CS_ROWS / 4);
        float4 v[CS_ROWS / 4];
#pragma unroll
        for (int j = 0; j < CS_ROWS / 4; ++j)
            v[j] = (c < cols_pad && r0 + j < rows) ? ld4(X + (r0 + j) * ld + c) : make_float4(0.f, 0.f, 0.f, 0.f);
        const float4 g = add4(add4(v[0], v[1]), add4(v[2], v[3]));
        acc = it == 0 ? g : add4(acc, g);
    }
    red[w][lane] = acc;
    __syncthreads();
    if (w == 0 && c < cols_pad)
        *reinterpret_cast<float4 *>(ws + (int64_t)by * cols_pad + c) =
            add4(add4(red[0][lane], red[1][lane]), add4(red[2][lane], red[3][lane]));
}

template <bool FOLD>
__global__ void __launch_bounds__(256) colsum_partial_kernel(const float *X, int64_t rows, int64_t cols_pad,
                                                             int64_t ld, int rep, float *ws) {
    colsum_partial_body<FOLD>(X, rows, cols_pad, ld, rep, ws, blockIdx.x, blockIdx.y);
}

// the same partial sums for operands that are not float4-addressable (e.g. a column vector):
// lane = column, wave w sums rows r0 + w*CS_ROWS/4 ...
__global__ void __launch_bounds__(256) colsum_partial_scalar_kernel(const float *X, int64_t rows, int64_t cols_pad,
                                                                    int64_t ld, float *ws) {
    __shared__ float red[4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t c = (int64_t)blockIdx.x * 64 + lane;
    const int64_t r0 = (int64_t)blockIdx.y * CS_ROWS + w * (CS_ROWS / 4);
    float v[CS_ROWS / 4];
#pragma unroll
    for (int j = 0; j < CS_ROWS / 4; ++j) v[j] = (c < cols_pad && r0 + j < rows) ? X[(r0 + j) * ld + c] : 0.f;
    red[w][lane] = (v[0] + v[1]) + (v[2] + v[3]);
    __syncthreads();
    if (w == 0 && c < cols_pad)
        ws[(int64_t)blockIdx.y * cols_pad + c] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}

// Single-launch column sums for short inputs (rows <= SMALL_ROWS: the ~100-node batches of C2 / C3,
// whose steps are latency-bound at ~5 us per launch): block = 1024 threads = 16 float4 columns x 64
// row lanes, lane l sums rows l, l+64, ... (2 accumulators), then a fixed-order LDS tree over the 64
// lanes (deterministic).  One block per 64 columns.  Measured slower at C5's 1920 rows (one CU per
// 64 columns reads too slowly there), hence the bound.
constexpr int64_t SMALL_ROWS = 512;

__device__ __forceinline__ void colsum_small_body(const float *X, int64_t rows, int64_t cols_pad, int64_t ld, int64_t cbp,
                                                  int64_t cbr, float *out, int accumulate, int bx) {
    __shared__ float4 red[64][16];
    const int cg = threadIdx.x & 15, rl = threadIdx.x >> 4;
    const int64_t c = ((int64_t)bx * 16 + cg) * 4;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 a = z4, b = z4;
    if (c < cols_pad) {
        int64_t r = rl;
        for (; r + 64 < rows; r += 128) {
            a = add4(a, ld4(X + r * ld + c));
            b = add4(b, ld4(X + (r + 64) * ld + c));
        }
        if (r < rows) a = add4(a, ld4(X + r * ld + c));
    }
    red[rl][cg] = add4(a, b);
#pragma unroll
    for (int h = 32; h > 0; h >>= 1) {
        __syncthreads();
        if (rl < h) red[rl][cg] = add4(red[rl][cg], red[rl + h][cg]);
    }
    __syncthreads();
    if (rl != 0 || c >= cols_pad) return;
    const float t[4] = {red[0][cg].x, red[0][cg].y, red[0][cg].z, red[0][cg].w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        bool v;
        const int64_t cc = blk_map(c + q, cbp, cbr, &v);
        if (v) out[cc] = accumulate ? out[cc] + t[q] : t[q];
    }
}

__global__ void __launch_bounds__(1024) colsum_small_kernel(const float *X, int64_t rows, int64_t cols_pad, int64_t ld,
                                                            int64_t cbp, int64_t cbr, float *out, int accumulate) {
    colsum_small_body(X, rows, cols_pad, ld, cbp, cbr, out, accumulate, blockIdx.x);
}

// stage 2: block = 16 columns x 16 chunk strides (thread t: column t%16, chunks t/16, t/16+16, ...),
// then a fixed-order LDS combine (deterministic).  ~cols/16 blocks keep the serial chain short.
constexpr int FIN_COLS = 16;

__device__ __forceinline__ void colsum_final_body(const float *ws, int64_t n_chunks, int64_t cols_pad, int64_t cbp,
                                                  int64_t cbr, float *out, int accumulate, int bx) {
    __shared__ float red[16][FIN_COLS + 1];
    const int cl = threadIdx.x % FIN_COLS, kg = threadIdx.x / FIN_COLS;
    const int64_t c = (int64_t)bx * FIN_COLS + cl;
    float s[2] = {0.f, 0.f};
    if (c < cols_pad) {
        // chunks kg, kg+16, kg+32, ... alternate between s[0] and s[1]; 8 loads in flight
        int64_t k = kg;
        for (; k + 112 < n_chunks; k += 128) {
            float l[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) l[q] = ws[(k + 16 * q) * cols_pad + c];
#pragma unroll
            for (int q = 0; q < 8; ++q) s[q & 1] += l[q];
        }
        for (; k + 16 < n_chunks; k += 32) {
            s[0] += ws[k * cols_pad + c];
            s[1] += ws[(k + 16) * cols_pad + c];
        }
        for (; k < n_chunks; k += 16) s[0] += ws[k * cols_pad + c];
    }
    red[kg][cl] = s[0] + s[1];
    __syncthreads();
    if (kg != 0 || c >= cols_pad) return;
    bool v;
    const int64_t cc = blk_map(c, cbp, cbr, &v);
    if (!v) return;
    float t = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) t += red[j][cl];
    out[cc] = accumulate ? out[cc] + t : t;
}

__global__ void __launch_bounds__(256) colsum_final_kernel(const float *ws, int64_t n_chunks, int64_t cols_pad,
                                                           int64_t cbp, int64_t cbr, float *out, int accumulate) {
    colsum_final_body(ws, n_chunks, cols_pad, cbp, cbr, out, accumulate, blockIdx.x);
}

// ------------------------------------------------------------------------------------------
// a3.2 attention probabilities: row softmax over the n_valid keys, dropout(p) on the
// probabilities (torch SDPA math path: dropout AFTER softmax, 1/(1-p) scaling).
// One 256-thread block per row; online max/sum pass, then normalise + mask pass.
// ------------------------------------------------------------------------------------------
// 8 bits -> bit 4i for bit i (the keep decisions of 8 lanes x 4 columns -> one 32-bit word)
__device__ __forceinline__ uint32_t spread4(uint32_t x) {
    x &= 0xFFu;
    x = (x | (x << 12)) & 0x000F000Fu;
    x = (x | (x << 6)) & 0x03030303u;
    x = (x | (x << 3)) & 0x11111111u;
    return x;
}

// One 256-thread block per row.  The row (n_pad <= 1024 * RV columns) is read ONCE into
// registers: block max, then e = exp(s - max) and its block sum (one exp per element), then P,
// Pd and the keep bits are written from the registers.  RV = float4 per thread: 8, 16 or 32
// (rows of up to 8192 / 16384 / 32768 keys).
constexpr int SM_RV_MAX = 32;

__device__ __forceinline__ float block_max4(float v, float *red, int lane, int w) {
    v = wave_max(v);
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    return fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

__device__ __forceinline__ float block_sum4(float v, float *red, int lane, int w) {
    v = wave_sum(v);
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    return (red[0] + red[1]) + (red[2] + red[3]);
}

template <int SM_RV>
__global__ void __launch_bounds__(256) attn_softmax_kernel(const float *S, int64_t lds, float *P, float *Pd,
                                                           int64_t ldp, int64_t rows_valid, int64_t n_valid,
                                                           int64_t n_pad, float p, uint64_t seed, const uint64_t *seed_epoch, uint32_t *keep,
                                                           int64_t ld_keep) {
    seed = u2gnn_seed(seed, seed_epoch);
    __shared__ float red[4];
    const int64_t row = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    // P == nullptr: signed image only, Pd = kept ? P/(1-p) : -P (the sign bit is the keep bit)
    const bool sgn = P == nullptr;
    float *prow = sgn ? nullptr : P + row * ldp;
    float *pdrow = Pd + row * ldp;
    uint32_t *krow = keep ? keep + row * ld_keep : nullptr;
    const bool write_pd = Pd != P;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    if (row >= rows_valid) {
        for (int64_t c = tid * 4; c < n_pad; c += 1024) {
            if (!sgn) *reinterpret_cast<float4 *>(prow + c) = z4;
            if (write_pd) *reinterpret_cast<float4 *>(pdrow + c) = z4;
        }
        if (krow)
            for (int64_t k = tid; k < n_pad / 32; k += 256) krow[k] = 0u;
        return;
    }
    const float *srow = S + row * lds;
    float e[SM_RV][4];
    float m = -INFINITY;
#pragma unroll
    for (int i = 0; i < SM_RV; ++i) {
        const int64_t c = (int64_t)i * 1024 + tid * 4;
        const float4 v = c < n_pad ? *reinterpret_cast<const float4 *>(srow + c) : z4;
        const float x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            e[i][j] = c + j < n_valid ? x[j] : -INFINITY;
            m = fmaxf(m, e[i][j]);
        }
    }
    const float M = block_max4(m, red, lane, w);
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < SM_RV; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            e[i][j] = expf(e[i][j] - M);   // exp(-inf) = 0 for masked / padded keys
            s += e[i][j];
        }
    const float inv = 1.f / block_sum4(s, red, lane, w);
    const float ks = p > 0.f ? 1.f / (1.f - p) : 1.f;
    const uint32_t rkey = u2gnn_row_key(seed, (uint32_t)row), thr = u2gnn_keep_thr(p);
#pragma unroll
    for (int i = 0; i < SM_RV; ++i) {
        const int64_t cb = (int64_t)i * 1024;
        if (cb >= n_pad) break;   // block-uniform
        const int64_t c = cb + tid * 4;
        const bool in = c < n_pad;
        float pv[4], pdv[4];
        bool kp[4];
        // one finaliser per column pair (c % 4 == 0: pairs c / 2 and c / 2 + 1), the same bits as u2gnn_keep_rk per
        // column (round 6: the per-column form hashed every pair twice; the hash's two quarter-rate multiplies made
        // it a third of this kernel's VALU issue)
        const uint32_t h0 = u2gnn_pair_hash(rkey, (uint32_t)(c >> 1)), h1 = u2gnn_pair_hash(rkey, (uint32_t)(c >> 1) + 1u);
        kp[0] = u2gnn_keep_lo(h0, thr), kp[1] = u2gnn_keep_hi(h0, thr);
        kp[2] = u2gnn_keep_lo(h1, thr), kp[3] = u2gnn_keep_hi(h1, thr);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            pv[j] = e[i][j] * inv;
            pdv[j] = kp[j] ? pv[j] * ks : (sgn ? -pv[j] : 0.f);
        }
        if (in) {
            if (!sgn) *reinterpret_cast<float4 *>(prow + c) = make_float4(pv[0], pv[1], pv[2], pv[3]);
            if (write_pd) *reinterpret_cast<float4 *>(pdrow + c) = make_float4(pdv[0], pdv[1], pdv[2], pdv[3]);
        }
        if (krow) {
            // lanes 8k..8k+7 cover columns 32k..32k+31 of this wave's 256: word k from 4 ballots
            uint32_t word = 0u;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint64_t b = __ballot(in && kp[j] && c + j < n_valid);
                word |= spread4((uint32_t)(b >> (8 * (lane & 7)))) << j;
            }
            if (lane < 8 && (cb + w * 256 + 32 * lane) < n_pad) krow[(cb + w * 256) / 32 + lane] = word;
        }
    }
}

// fp32 -> x2 over rows x cols (cols % 4 == 0): one thread per 4 columns
__global__ void __launch_bounds__(256) split_x2_kernel(const float *src, int64_t ld_src, __bf16 *dst, int64_t ld_dst,
                                                       int64_t rows, int64_t cols) {
    const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x, per = cols / 4;
    if (q >= rows * per) return;
    const int64_t r = q / per, c = (q - r * per) * 4;
    store_x2_4(dst, ld_dst, (int)r, (int)c, *reinterpret_cast<const float4 *>(src + r * ld_src + c));
}

__global__ void __launch_bounds__(256) rowdot_kernel(const float *A, int64_t lda, const float *B, int64_t ldb,
                                                     float *out, int64_t rows, int64_t cols) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= rows) return;
    float s = 0.f;
    for (int64_t c = lane; c < cols; c += 64) s += A[row * lda + c] * B[row * ldb + c];
    s = wave_sum(s);
    if (lane == 0) out[row] = s;
}

// ------------------------------------------------------------------------------------------
// a3.3/a3.4 post-LN (eps 1e-5).  One half-wave (32 lanes) per row, a float4 of columns per lane,
// the row cached in registers (d_pad <= 1024): 16-byte loads/stores, 8 rows per block.
// ------------------------------------------------------------------------------------------
constexpr int LN_V4_MAX = 8;   // d_pad / 128 upper bound (template V4: float4 per lane = ceil(d_pad / 128))
constexpr int LN_MAXV = 16;    // d_pad / 64 upper bound (host check)

__device__ __forceinline__ float half_sum(float v) {
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// sum over the LPR lanes (32: a half-wave, 64: a wave) that hold one row
template <int LPR>
__device__ __forceinline__ float row_sum(float v) {
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

template <int LN_V4, int LPR = 32>
__global__ void __launch_bounds__(256) layernorm_fwd_kernel(const float *Z, int64_t ldz, const float *gamma,
                                                            const float *beta, float *Y, int64_t ldy, float *mean,
                                                            float *rstd, int64_t rows_valid, int64_t rows_pad,
                                                            int64_t d, int64_t d_pad, float eps) {
    const int64_t row = (int64_t)blockIdx.x * (256 / LPR) + (threadIdx.x / LPR);   // LPR lanes per row
    const int hl = threadIdx.x & (LPR - 1);
    if (row >= rows_pad) return;
    float *y = Y + row * ldy;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    if (row >= rows_valid) {
        for (int64_t c = hl * 4; c < d_pad; c += 4 * LPR) *reinterpret_cast<float4 *>(y + c) = z4;
        if (hl == 0) {
            mean[row] = 0.f;
            rstd[row] = 0.f;
        }
        return;
    }
    const float *z = Z + row * ldz;
    float v[LN_V4][4], gm[LN_V4][4] = {}, bt[LN_V4][4] = {};
    float4 t[LN_V4];
#pragma unroll
    for (int i = 0; i < LN_V4; ++i) {
        const int64_t c = 4 * (hl + LPR * i);
        t[i] = c < d_pad ? ld4(z + c) : z4;
    }
    // gamma / beta are unpadded [d] vectors: element loads at a clamped column, issued with the row's
    // loads (no per-element branch, no second round trip later) -- or, when both are 16-byte aligned
    // (the flat parameter buffer's views are), one float4 per full 4-column chunk
    const bool gb16 = ((reinterpret_cast<uintptr_t>(gamma) | reinterpret_cast<uintptr_t>(beta)) & 15) == 0;
#pragma unroll
    for (int i = 0; i < LN_V4; ++i) {
        const int64_t c = 4 * (hl + LPR * i);
        if (c >= d_pad) continue;
        if (gb16 && c + 4 <= d) {
            const float4 g = ld4(gamma + c), b = ld4(beta + c);
            gm[i][0] = g.x, gm[i][1] = g.y, gm[i][2] = g.z, gm[i][3] = g.w;
            bt[i][0] = b.x, bt[i][1] = b.y, bt[i][2] = b.z, bt[i][3] = b.w;
            continue;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int64_t cc = c + q < d ? c + q : d - 1;
            gm[i][q] = gamma[cc];
            bt[i][q] = beta[cc];
        }
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < LN_V4; ++i) {
        const int64_t c = 4 * (hl + LPR * i);
        const float x[4] = {t[i].x, t[i].y, t[i].z, t[i].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            v[i][q] = c + q < d ? x[q] : 0.f;
            s += v[i][q];
        }
    }
    const float mu = row_sum<LPR>(s) / (float)d;
    float sq = 0.f;
#pragma unroll
    for (int i = 0; i < LN_V4; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float t = 4 * (hl + LPR * i) + q < d ? v[i][q] - mu : 0.f;
            sq += t * t;
        }
    const float rs = rsqrtf(row_sum<LPR>(sq) / (float)d + eps);
#pragma unroll
    for (int i = 0; i < LN_V4; ++i) {
        const int64_t c = 4 * (hl + LPR * i);
        if (c >= d_pad) continue;
        float o[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = c + q < d ? (v[i][q] - mu) * rs * gm[i][q] + bt[i][q] : 0.f;
        *reinterpret_cast<float4 *>(y + c) = make_float4(o[0], o[1], o[2], o[3]);
    }
    if (hl == 0) {
        mean[row] = mu;
        rstd[row] = rs;
    }
}

// LN backward, row part: one half-wave per row (8 rows per block).
// DELTA (LayerNorm1 of an encoder layer, u2gnn_layernorm_bwd_delta): also the attention backward's
// delta[row] = sum_c dZd[row,c] * ((Z - X)[row,c] * (1-p) - bias[c]).  Z = X + drop(A + bias) with
// A = O W_o^T the out-projection product, so where dZd != 0 (kept) the bracket is A, and
// sum_c dZd * A = sum_c (dZd W_o) * O = rowsum(dO * O): the u2gnn_rowdot launch without reading dO / O.
struct LnDelta {
    const float *X;
    int64_t ldx;
    const float *bias;   // [d_pad], zero-padded (the out-projection's padded bias)
    float *delta;        // [rows_pad]
    // SLABS (u2gnn_layernorm_bwd_delta_slabs): dY += the split-K slabs of the FFN's dX1 product first
    // (slab_sum4's order, the result written back to dY: u2gnn_slab_reduce accumulate fused in)
    const float *slabs;
    int64_t slab_stride;
    int n_slab;
};

template <int LN_V4, bool DELTA, bool SLABS = false>
__global__ void __launch_bounds__(256) layernorm_bwd_kernel(const float *dY, int64_t ldy, const float *Z, int64_t ldz,
                                                            const float *mean, const float *rstd, const float *gamma,
                                                            float *dZ, int64_t lddz, float *dZd, int64_t lddrop,
                                                            float p, uint64_t seed, const uint64_t *seed_epoch, int64_t rows_valid,
                                                            int64_t rows_pad, int64_t d, int64_t d_pad, LnDelta dt) {
    seed = u2gnn_seed(seed, seed_epoch);
    const int64_t row = (int64_t)blockIdx.x * 8 + (threadIdx.x >> 5);
    const int hl = threadIdx.x & 31;
    if (row >= rows_pad) return;
    float *dz = dZ + row * lddz;
    float *dzd = dZd ? dZd + row * lddrop : nullptr;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    if (row >= rows_valid) {
        for (int64_t c = hl * 4; c < d_pad; c += 128) {
            *reinterpret_cast<float4 *>(dz + c) = z4;
            if (dzd) *reinterpret_cast<float4 *>(dzd + c) = z4;
        }
        if constexpr (DELTA)
            if (hl == 0) dt.delta[row] = 0.f;
        return;
    }
    const float ks = p > 0.f ? 1.f / (1.f - p) : 1.f;
    const float mu = mean[row], rs = rstd[row];
    const float *dy = dY + row * ldy;
    const float *z = Z + row * ldz;
    float xh[LN_V4][4], g[LN_V4][4], gm[LN_V4][4] = {};
    float4 ta[LN_V4], tb[LN_V4], tx[DELTA ? LN_V4 : 1], tc[DELTA ? LN_V4 : 1];
#pragma unroll
    for (int i = 0; i < LN_V4; ++i) {
        const int64_t c = 4 * (hl + 32 * i);
        ta[i] = c < d_pad ? ld4(dy + c) : z4;
        tb[i] = c < d_pad ? ld4(z + c) : z4;
        if constexpr (SLABS) {
            if (c < d_pad) {
                ta[i] = add4(slab_sum4(dt.slabs + row * ldy + c, dt.n_slab, dt.slab_stride), ta[i]);
                *reinterpret_cast<float4 *>(const_cast<float *>(dy) + c) = ta[i];
            }
        }
        if constexpr (DELTA) {
            tx[i] = c < d_pad ? ld4(dt.X + row * dt.ldx + c) : z4;
            tc[i] = c < d_pad ? ld4(dt.bias + c) : z4;
        }
    }
    const bool g16 = (reinterpret_cast<uintptr_t>(gamma) & 15) == 0;
#pragma unroll
    for (int i = 0; i < LN_V4; ++i) {   // unpadded [d] gamma: float4 or clamped element loads (see the forward)
        const int64_t c = 4 * (hl + 32 * i);
        if (c >= d_pad) continue;
        if (g16 && c + 4 <= d) {
            const float4 g = ld4(gamma + c);
            gm[i][0] = g.x, gm[i][1] = g.y, gm[i][2] = g.z, gm[i][3] = g.w;
            continue;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) gm[i][q] = gamma[c + q < d ? c + q : d - 1];
    }
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < LN_V4; ++i) {
        const int64_t c = 4 * (hl + 32 * i);
        const float av[4] = {ta[i].x, ta[i].y, ta[i].z, ta[i].w}, bv[4] = {tb[i].x, tb[i].y, tb[i].z, tb[i].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const bool ok = c + q < d;
            xh[i][q] = ok ? (bv[q] - mu) * rs : 0.f;
            g[i][q] = ok ? av[q] * gm[i][q] : 0.f;
            s1 += g[i][q];
            s2 += g[i][q] * xh[i][q];
        }
    }
    const float m1 = half_sum(s1) / (float)d;
    const float m2 = half_sum(s2) / (float)d;
    float s3 = 0.f;   // DELTA
#pragma unroll
    for (int i = 0; i < LN_V4; ++i) {
        const int64_t c = 4 * (hl + 32 * i);
        if (c >= d_pad) continue;
        float o[4], od[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const bool ok = c + q < d;
            o[q] = ok ? rs * (g[i][q] - m1 - xh[i][q] * m2) : 0.f;
            od[q] = (ok && p > 0.f) ? (u2gnn_keep(seed, (uint32_t)row, (uint32_t)(c + q), p) ? o[q] * ks : 0.f) : o[q];
        }
        *reinterpret_cast<float4 *>(dz + c) = make_float4(o[0], o[1], o[2], o[3]);
        if (dzd) *reinterpret_cast<float4 *>(dzd + c) = make_float4(od[0], od[1], od[2], od[3]);
        if constexpr (DELTA) {
            const float zv[4] = {tb[i].x, tb[i].y, tb[i].z, tb[i].w}, xv[4] = {tx[i].x, tx[i].y, tx[i].z, tx[i].w};
            const float bv[4] = {tc[i].x, tc[i].y, tc[i].z, tc[i].w};
#pragma unroll
            for (int q = 0; q < 4; ++q) s3 += od[q] * ((zv[q] - xv[q]) * (1.f - p) - bv[q]);
        }
    }
    if constexpr (DELTA) {
        const float dl = half_sum(s3);
        if (hl == 0) dt.delta[row] = dl;
    }
}

// LN backward, column part: per CS_ROWS-row chunk, sums over rows of dY*xhat (dgamma), dY (dbeta)
// and dZd (the bias gradient of the dropout branch feeding this LN) -> ws[chunk][3][d_pad];
// float4 columns per lane, CS_ROWS/4 rows per wave (all loads in flight); a chunk spans rep
// consecutive CS_ROWS-row groups so that token-sized inputs (neighbour mode, ~82K rows) leave few
// enough chunks for ln_param_reduce's column-parallel combine (rep = 1 below 8K rows).
template <bool FOLD>
__device__ __forceinline__ void ln_colstats_body(const float *dY, int64_t ldy, const float *Z, int64_t ldz,
                                                 const float *mean, const float *rstd, const float *dZd, int64_t lddrop,
                                                 int64_t rows, int64_t d_pad, int rep, float *ws, int bx, int by) {
    __shared__ float4 red[4][3][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t c = ((int64_t)bx * 64 + lane) * 4;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 sg = z4, sb = z4, sd = z4;
    const int nrep = FOLD ? rep : 1;
    for (int it = 0; it < nrep && c < d_pad; ++it) {
        const int64_t r0 = ((int64_t)by * nrep + it) * CS_ROWS + w * (CS_ROWS / 4);
        float4 dy[CS_ROWS / 4], zz[CS_ROWS / 4], dd[CS_ROWS / 4];
        float mu[CS_ROWS / 4], rs[CS_ROWS / 4];
#pragma unroll
        for (int j = 0; j < CS_ROWS / 4; ++j) {
            const int64_t r = r0 + j;
            const bool ok = r < rows;
            dy[j] = ok ? ld4(dY + r * ldy + c) : z4;
            zz[j] = ok ? ld4(Z + r * ldz + c) : z4;
            dd[j] = (ok && dZd) ? ld4(dZd + r * lddrop + c) : z4;
            mu[j] = ok ? mean[r] : 0.f;
            rs[j] = ok ? rstd[r] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < CS_ROWS / 4; ++j) {
            sg.x += dy[j].x * ((zz[j].x - mu[j]) * rs[j]);
            sg.y += dy[j].y * ((zz[j].y - mu[j]) * rs[j]);
            sg.z += dy[j].z * ((zz[j].z - mu[j]) * rs[j]);
            sg.w += dy[j].w * ((zz[j].w - mu[j]) * rs[j]);
            sb = add4(sb, dy[j]);
            sd = add4(sd, dd[j]);
        }
    }
    red[w][0][lane] = sg;
    red[w][1][lane] = sb;
    red[w][2][lane] = sd;
    __syncthreads();
    if (w < 3 && c < d_pad)
        *reinterpret_cast<float4 *>(ws + ((int64_t)by * 3 + w) * d_pad + c) =
            add4(add4(red[0][w][lane], red[1][w][lane]), add4(red[2][w][lane], red[3][w][lane]));
}

template <bool FOLD>
__global__ void __launch_bounds__(256) ln_colstats_kernel(const float *dY, int64_t ldy, const float *Z, int64_t ldz,
                                                          const float *mean, const float *rstd, const float *dZd,
                                                          int64_t lddrop, int64_t rows, int64_t d, int64_t d_pad,
                                                          int rep, float *ws) {
    (void)d;
    ln_colstats_body<FOLD>(dY, ldy, Z, ldz, mean, rstd, dZd, lddrop, rows, d_pad, rep, ws, blockIdx.x, blockIdx.y);
}

constexpr int64_t LN_MAX_CHUNKS = 512;

// single-launch LN parameter gradients for short inputs (rows <= SMALL_ROWS), the layout of
// colsum_small_kernel with three sums (dY * xhat, dY, dZd)
__device__ __forceinline__ void ln_params_small_body(const float *dY, int64_t ldy, const float *Z, int64_t ldz,
                                                     const float *mean, const float *rstd, const float *dZd,
                                                     int64_t lddrop, int64_t rows, int64_t d, int64_t d_pad,
                                                     float *dgamma, float *dbeta, float *dbias, int bx) {
    __shared__ float4 red[3][64][16];
    const int cg = threadIdx.x & 15, rl = threadIdx.x >> 4;
    const int64_t c = ((int64_t)bx * 16 + cg) * 4;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 sg = z4, sb = z4, sd = z4;
    if (c < d_pad) {
        for (int64_t r = rl; r < rows; r += 64) {
            const float4 dy = ld4(dY + r * ldy + c), zz = ld4(Z + r * ldz + c);
            const float4 dd = dZd ? ld4(dZd + r * lddrop + c) : z4;
            const float mu = mean[r], rs = rstd[r];
            sg.x += dy.x * ((zz.x - mu) * rs);
            sg.y += dy.y * ((zz.y - mu) * rs);
            sg.z += dy.z * ((zz.z - mu) * rs);
            sg.w += dy.w * ((zz.w - mu) * rs);
            sb = add4(sb, dy);
            sd = add4(sd, dd);
        }
    }
    red[0][rl][cg] = sg;
    red[1][rl][cg] = sb;
    red[2][rl][cg] = sd;
#pragma unroll
    for (int h = 32; h > 0; h >>= 1) {
        __syncthreads();
        if (rl < h)
#pragma unroll
            for (int k = 0; k < 3; ++k) red[k][rl][cg] = add4(red[k][rl][cg], red[k][rl + h][cg]);
    }
    __syncthreads();
    if (rl != 0) return;
    const float4 g = red[0][0][cg], b = red[1][0][cg], e = red[2][0][cg];
    const float gv[4] = {g.x, g.y, g.z, g.w}, bv[4] = {b.x, b.y, b.z, b.w}, ev[4] = {e.x, e.y, e.z, e.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        if (c + q >= d) break;
        dgamma[c + q] = gv[q];
        dbeta[c + q] = bv[q];
        if (dbias) dbias[c + q] = ev[q];
    }
}

__global__ void __launch_bounds__(1024) ln_params_small_kernel(const float *dY, int64_t ldy, const float *Z, int64_t ldz,
                                                               const float *mean, const float *rstd, const float *dZd,
                                                               int64_t lddrop, int64_t rows, int64_t d, int64_t d_pad,
                                                               float *dgamma, float *dbeta, float *dbias) {
    ln_params_small_body(dY, ldy, Z, ldz, mean, rstd, dZd, lddrop, rows, d, d_pad, dgamma, dbeta, dbias, blockIdx.x);
}

// block = 16 columns x 16 chunk strides (as colsum_final), fixed-order LDS combine
__device__ __forceinline__ void ln_param_reduce_body(const float *ws, int64_t n_chunks, int64_t d, int64_t d_pad,
                                                     float *dgamma, float *dbeta, float *dbias, int bx) {
    __shared__ float red[3][16][FIN_COLS + 1];
    const int cl = threadIdx.x % FIN_COLS, kg = threadIdx.x / FIN_COLS;
    const int64_t c = (int64_t)bx * FIN_COLS + cl;
    float a = 0.f, b = 0.f, e = 0.f;
    if (c < d) {
        int64_t k = kg;
        for (; k + 48 < n_chunks; k += 64) {   // 12 loads in flight, same add order
            float l[4][3];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float *q = ws + (k + 16 * j) * 3 * d_pad + c;
                l[j][0] = q[0], l[j][1] = q[d_pad], l[j][2] = q[2 * d_pad];
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) a += l[j][0], b += l[j][1], e += l[j][2];
        }
        for (; k < n_chunks; k += 16) {
            const float *q = ws + k * 3 * d_pad + c;
            a += q[0];
            b += q[d_pad];
            e += q[2 * d_pad];
        }
    }
    red[0][kg][cl] = a;
    red[1][kg][cl] = b;
    red[2][kg][cl] = e;
    __syncthreads();
    if (kg != 0 || c >= d) return;
    float t[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        t[0] += red[0][j][cl];
        t[1] += red[1][j][cl];
        t[2] += red[2][j][cl];
    }
    dgamma[c] = t[0];
    dbeta[c] = t[1];
    if (dbias) dbias[c] = t[2];
}

__global__ void __launch_bounds__(256) ln_param_reduce_kernel(const float *ws, int64_t n_chunks, int64_t d,
                                                              int64_t d_pad, float *dgamma, float *dbeta, float *dbias) {
    ln_param_reduce_body(ws, n_chunks, d, d_pad, dgamma, dbeta, dbias, blockIdx.x);
}

// ------------------------------------------------------------------------------------------
// a3.4 for d <= 256 encoders whose FFN2 product has too few output tiles to fill the chip (C5: 32
// row-complete 64x64 tiles; C2's IMDBBINARY batches: 4): the product runs split-K into slabs, and this
// pass sums the slabs (slab_reduce's order), adds the bias, applies dropout (the GEMM epilogue's hash)
// and the residual -> Z, then the row's LayerNorm (two-pass mean / mean square deviation over the first
// d columns) -> Y, mean, rstd.  One wave per row; lane l holds columns l, l + 64, ... (CPL = dp / 64 of
// them, coalesced per wave); at CPL = 1 the sums are the round-4 kernel's, term for term.
// ------------------------------------------------------------------------------------------
template <int CPL>
__global__ void __launch_bounds__(256) slab_bias_drop_resid_ln_kernel(
    const float *src, int n_slab, int64_t slab_stride, int64_t ld_src, const float *bias, const float *resid,
    int64_t ld_res, float p, uint64_t seed, const uint64_t *seed_epoch, float *Z, int64_t ldz, const float *gamma,
    const float *beta, float *Y, int64_t ldy, float *mean, float *rstd, int64_t d, int64_t rows_valid,
    int64_t rows_pad, float eps) {
    seed = u2gnn_seed(seed, seed_epoch);
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int l = threadIdx.x & 63;
    if (row >= rows_pad) return;
    const bool live = row < rows_valid;   // padding rows: Z, Y, mean, rstd all 0
    // the column groups' loads of one 4-slab round issued together, bias and residual before the rounds (round 6:
    // a round per column group, then the remainder slab by slab, each waited out a memory round trip,
    // tools/isa_waits.py); the sums per column are the same, in the same order
    float zz[CPL], a[CPL], b[CPL], e[CPL], f[CPL], bi[CPL], re[CPL], gm[CPL], bt[CPL];
    const float *q = src + row * ld_src + l;
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
        const int cc = l + 64 * k < d ? l + 64 * k : (int)d - 1;
        a[k] = b[k] = e[k] = f[k] = 0.f;
        bi[k] = bias[l + 64 * k];
        re[k] = resid[row * ld_res + l + 64 * k];
        gm[k] = gamma[cc], bt[k] = beta[cc];
    }
    int z = 0;
    for (; z + 4 <= n_slab; z += 4) {
        float t[CPL][4];
#pragma unroll
        for (int k = 0; k < CPL; ++k)
#pragma unroll
            for (int j = 0; j < 4; ++j) t[k][j] = q[(int64_t)(z + j) * slab_stride + 64 * k];
#pragma unroll
        for (int k = 0; k < CPL; ++k) a[k] += t[k][0], b[k] += t[k][1], e[k] += t[k][2], f[k] += t[k][3];
    }
    if (z < n_slab) {   // the last 1-3 slabs: clamped loads together, then added in slab order
        const int z1 = min(z + 1, n_slab - 1), z2 = min(z + 2, n_slab - 1);
        float t[CPL][3];
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
            t[k][0] = q[(int64_t)z * slab_stride + 64 * k];
            t[k][1] = q[(int64_t)z1 * slab_stride + 64 * k];
            t[k][2] = q[(int64_t)z2 * slab_stride + 64 * k];
        }
#pragma unroll
        for (int k = 0; k < CPL; ++k)   // (consumed here: keeps the compiler from sinking a load into its branch)
            asm volatile("" ::"v"(t[k][0]), "v"(t[k][1]), "v"(t[k][2]));
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
            a[k] += t[k][0];
            if (z + 1 < n_slab) a[k] += t[k][1];
            if (z + 2 < n_slab) a[k] += t[k][2];
        }
    }
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < CPL; ++k) asm volatile("" ::"v"(gm[k]), "v"(bt[k]));   // (loaded with the slabs: see above)
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
        const int c = l + 64 * k;
        float x = ((a[k] + b[k]) + (e[k] + f[k])) + bi[k];
        if (p > 0.f) x = u2gnn_keep(seed, (uint32_t)row, (uint32_t)c, p) ? x * (1.f / (1.f - p)) : 0.f;
        zz[k] = x + re[k];
        Z[row * ldz + c] = live ? zz[k] : 0.f;
        s += c < d ? zz[k] : 0.f;
    }
    const float mu = wave_sum(s) / (float)d;
    float q2 = 0.f;
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
        const float t = l + 64 * k < d ? zz[k] - mu : 0.f;
        q2 += t * t;
    }
    const float rs = rsqrtf(wave_sum(q2) / (float)d + eps);
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
        const int c = l + 64 * k;
        Y[row * ldy + c] = (live && c < d) ? (zz[k] - mu) * rs * gm[k] + bt[k] : 0.f;
    }
    if (l == 0) {
        mean[row] = live ? mu : 0.f;
        rstd[row] = live ? rs : 0.f;
    }
}

// ------------------------------------------------------------------------------------------
// batched reductions (u2gnn_reduce_batch): the jobs of one launch travel by value in the kernel
// arguments; a block finds its job by walking the per-job block counts (uniform, scalar) and runs
// that job's body with its own block coordinates.  Latency-bound layers (C5: ~4.6 us per launch of
// a few-KB reduction) issue a layer's 8-12 reductions as 2 launches.
// ------------------------------------------------------------------------------------------
enum RbKind : int32_t { RB_SLAB, RB_CS_PART, RB_CS_FINAL, RB_CS_SMALL, RB_LN_PART, RB_LN_FINAL, RB_LN_SMALL };
constexpr int RB_MAX = 12;
struct RbJob {
    int32_t kind, nblk, nbx, n;   // n: slab count / fold rep / chunk count
    int32_t flag, vec;            // accumulate; vectorised slab store
    float alpha;
    const float *src, *Z, *mean, *rstd, *dZd;
    float *o0, *o1, *o2, *ws;
    int64_t ld_src, stride, rows, cols, d, rbp, rbr, cbp, cbr, ld_dst, ldz, lddrop;
};
struct RbBatch {
    RbJob j[RB_MAX];
    int32_t n;
};

template <int NT>
__global__ void __launch_bounds__(NT) reduce_batch_kernel(RbBatch B) {
    int bid = blockIdx.x, j = 0;
    while (j + 1 < B.n && bid >= B.j[j].nblk) bid -= B.j[j++].nblk;
    const RbJob &J = B.j[j];
    if constexpr (NT == 256) {
        switch (J.kind) {
            case RB_SLAB:
                slab_reduce_body(J.src, J.n, J.stride, J.rows, J.cols, J.ld_src, J.rbp, J.rbr, J.cbp, J.cbr, J.o0,
                                 J.ld_dst, J.alpha, J.flag, J.vec, (int64_t)bid * 256 + threadIdx.x);
                break;
            case RB_CS_PART:
                colsum_partial_body<true>(J.src, J.rows, J.cols, J.ld_src, J.n, J.ws, bid % J.nbx, bid / J.nbx);
                break;
            case RB_CS_FINAL: colsum_final_body(J.ws, J.n, J.cols, J.cbp, J.cbr, J.o0, J.flag, bid); break;
            case RB_LN_PART:
                ln_colstats_body<true>(J.src, J.ld_src, J.Z, J.ldz, J.mean, J.rstd, J.dZd, J.lddrop, J.rows, J.cols, J.n,
                                       J.ws, bid % J.nbx, bid / J.nbx);
                break;
            case RB_LN_FINAL: ln_param_reduce_body(J.ws, J.n, J.d, J.cols, J.o0, J.o1, J.o2, bid); break;
            default: break;
        }
    } else {
        switch (J.kind) {
            case RB_SLAB:
                slab_reduce_body(J.src, J.n, J.stride, J.rows, J.cols, J.ld_src, J.rbp, J.rbr, J.cbp, J.cbr, J.o0,
                                 J.ld_dst, J.alpha, J.flag, J.vec, (int64_t)bid * NT + threadIdx.x);
                break;
            case RB_CS_SMALL: colsum_small_body(J.src, J.rows, J.cols, J.ld_src, J.cbp, J.cbr, J.o0, J.flag, bid); break;
            case RB_LN_SMALL:
                ln_params_small_body(J.src, J.ld_src, J.Z, J.ldz, J.mean, J.rstd, J.dZd, J.lddrop, J.rows, J.d, J.cols,
                                     J.o0, J.o1, J.o2, bid);
                break;
            default: break;
        }
    }
}

__global__ void __launch_bounds__(256) dropout_mask_kernel(uint64_t seed, const uint64_t *seed_epoch, int64_t rows, int64_t cols, float p,
                                                           uint8_t *out) {
    seed = u2gnn_seed(seed, seed_epoch);
    const int64_t total = rows * cols;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        const int64_t r = i / cols, c = i - r * cols;
        out[i] = u2gnn_keep(seed, (uint32_t)r, (uint32_t)c, p) ? 1 : 0;
    }
}

__global__ void __launch_bounds__(256) dropout_kernel(const float *X, int64_t ldx, float *Y, int64_t ldy, int64_t rows,
                                                      int64_t cols, float p, uint64_t seed, const uint64_t *seed_epoch) {
    seed = u2gnn_seed(seed, seed_epoch);
    const int64_t total = rows * cols;
    const float ks = 1.f / (1.f - p);
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        const int64_t r = i / cols, c = i - r * cols;
        const float v = X[r * ldx + c];
        Y[r * ldy + c] = u2gnn_keep(seed, (uint32_t)r, (uint32_t)c, p) ? v * ks : 0.f;
    }
}

inline bool al16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

inline unsigned grid_for(int64_t n, int64_t per_block, int64_t cap = 8192) {
    int64_t g = (n + per_block - 1) / per_block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}

}  // namespace

extern "C" {

int u2gnn_gather_rows(const float *src, int64_t ld_src, int64_t src_rows, const int64_t *idx, int64_t idx_stride,
                      float *dst, int64_t ld_dst, int64_t n_rows, int64_t n_rows_pad, int64_t d, int64_t d_pad,
                      int32_t *err, void *stream) {
    if (!dst || (n_rows > 0 && (!src || !idx)) || n_rows > n_rows_pad || d > d_pad) return U2GNN_E_ARG;
    if (n_rows_pad == 0) return U2GNN_OK;
    const dim3 grid(grid_for(n_rows_pad, 4, 1 << 30));
    hipStream_t st = u2gnn_stream(stream);
    const bool small = d_pad <= 1024;
    if (small && (d_pad & 3) == 0 && (ld_dst & 3) == 0 && al16(dst) && (ld_src & 3) == 0 && al16(src))
        hipLaunchKernelGGL(gather_rows_kernel<1>, grid, dim3(256), 0, st, src, ld_src, src_rows, idx, idx_stride, dst,
                           ld_dst, n_rows, n_rows_pad, d, d_pad, err);
    else if (d_pad <= 512 && (ld_dst & 3) == 0 && al16(dst)) {
        // gridDim.x a multiple of 8 for the XCD order (surplus blocks find no rows and return)
        const dim3 g8((grid_for(n_rows_pad, 4, 1 << 30) + 7u) / 8u * 8u);
        if (d_pad & 3)
            hipLaunchKernelGGL((gather_rows_multi_kernel<1, false, true>), g8, dim3(256), 0, st, src, ld_src, src_rows,
                               idx, idx_stride, dst, ld_dst, n_rows, n_rows_pad, d, d_pad, err);
        else
            hipLaunchKernelGGL((gather_rows_multi_kernel<1, true, true>), g8, dim3(256), 0, st, src, ld_src, src_rows,
                               idx, idx_stride, dst, ld_dst, n_rows, n_rows_pad, d, d_pad, err);
    } else if (small)
        hipLaunchKernelGGL(gather_rows_kernel<2>, grid, dim3(256), 0, st, src, ld_src, src_rows, idx, idx_stride, dst,
                           ld_dst, n_rows, n_rows_pad, d, d_pad, err);
    else
        hipLaunchKernelGGL(gather_rows_kernel<0>, grid, dim3(256), 0, st, src, ld_src, src_rows, idx, idx_stride, dst,
                           ld_dst, n_rows, n_rows_pad, d, d_pad, err);
    return u2gnn_launch_status();
}

int u2gnn_scatter_add_rows(const float *src, int64_t ld_src, const int64_t *idx, int64_t idx_stride, float *dst,
                           int64_t ld_dst, int64_t dst_rows, int64_t n_rows, int64_t d, int32_t *err, void *stream) {
    if (n_rows == 0) return U2GNN_OK;
    if (!src || !idx || !dst || dst_rows < 0) return U2GNN_E_ARG;
    hipLaunchKernelGGL(scatter_add_rows_kernel, dim3(grid_for(n_rows, 4, 1 << 30)), dim3(256), 0,
                       u2gnn_stream(stream), src, ld_src, idx, idx_stride, dst, ld_dst, dst_rows, n_rows, d, err);
    return u2gnn_launch_status();
}

int u2gnn_slab_reduce(const float *src, int32_t n_slab, int64_t slab_stride, int64_t rows_pad, int64_t cols_pad,
                      int64_t ld_src, int64_t rblk_pad, int64_t rblk_real, int64_t cblk_pad, int64_t cblk_real,
                      float *dst, int64_t ld_dst, float alpha, int32_t accumulate, void *stream) {
    if (!src || !dst || n_slab < 1 || rblk_pad < 1 || cblk_pad < 1) return U2GNN_E_ARG;
    if (!al16(src) || (cols_pad & 3) || (ld_src & 3) || (slab_stride & 3)) return U2GNN_E_ALIGN;
    if (rows_pad == 0 || cols_pad == 0) return U2GNN_OK;
    const int vec_store = cblk_pad == cblk_real && al16(dst) && (ld_dst & 3) == 0;
    hipLaunchKernelGGL(slab_reduce_kernel, dim3(grid_for(rows_pad * (cols_pad / 4), 256, 1 << 30)), dim3(256), 0,
                       u2gnn_stream(stream), src, n_slab, slab_stride, rows_pad, cols_pad, ld_src, rblk_pad, rblk_real,
                       cblk_pad, cblk_real, dst, ld_dst, alpha, accumulate, vec_store);
    return u2gnn_launch_status();
}

int u2gnn_pack_padded(const float *src, int64_t ld_src, int64_t rows_pad, int64_t cols_pad, int64_t rblk_pad,
                      int64_t rblk_real, int64_t cblk_pad, int64_t cblk_real, float *dst, int64_t ld_dst,
                      void *stream) {
    if (!src || !dst || rblk_pad < 1 || cblk_pad < 1) return U2GNN_E_ARG;
    hipLaunchKernelGGL(pack_padded_kernel, dim3(grid_for(rows_pad * cols_pad, 256)), dim3(256), 0,
                       u2gnn_stream(stream), src, ld_src, rows_pad, cols_pad, rblk_pad, rblk_real, cblk_pad, cblk_real,
                       dst, ld_dst);
    return u2gnn_launch_status();
}

int u2gnn_pack_padded_multi(const u2gnn_pack_desc *descs, int32_t n, void *stream) {
    return u2gnn_pack_padded_multi_adv(descs, n, nullptr, nullptr, stream);
}

int u2gnn_pack_padded_multi_adv(const u2gnn_pack_desc *descs, int32_t n, uint64_t *epoch, int64_t *t,
                                void *stream) {
    if (n < 0 || (n && !descs)) return U2GNN_E_ARG;
    if (n == 0) return (epoch || t) ? U2GNN_E_ARG : U2GNN_OK;   // the advance needs a launch
    for (int32_t o = 0; o < n; o += PACK_MAX) {
        PackBatch pb;
        pb.adv_epoch = o == 0 ? epoch : nullptr;
        pb.adv_t = o == 0 ? t : nullptr;
        const int32_t m = n - o < PACK_MAX ? n - o : PACK_MAX;
        int64_t biggest = 1, max_rows = 1;
        bool fits32 = true;
        for (int32_t i = 0; i < m; ++i) {
            pb.d[i] = descs[o + i];
            const u2gnn_pack_desc &d = pb.d[i];
            if (!d.src || !d.dst || d.rblk_pad < 1 || d.cblk_pad < 1 || d.rows_pad < 0 || d.cols_pad < 0)
                return U2GNN_E_ARG;
            biggest = std::max<int64_t>(biggest, d.rows_pad * d.cols_pad);
            max_rows = std::max<int64_t>(max_rows, d.rows_pad);
            // 32-bit maps: padded extents, and the real row / column indices they map to
            const int64_t lim = (int64_t)1 << 31;
            fits32 = fits32 && d.rows_pad + d.rblk_pad < lim && d.cols_pad + d.cblk_pad < lim &&
                     d.rblk_real < lim && d.cblk_real < lim;
        }
        if (fits32)
            hipLaunchKernelGGL(pack_multi_kernel, dim3((unsigned)((max_rows + PACK_RB - 1) / PACK_RB), (unsigned)m),
                               dim3(256), 0, u2gnn_stream(stream), pb);
        else
            hipLaunchKernelGGL(pack_multi64_kernel, dim3(grid_for(biggest, 256, 2048), (unsigned)m), dim3(256), 0,
                               u2gnn_stream(stream), pb);
    }
    return u2gnn_launch_status();
}

int u2gnn_colsum(const float *X, int64_t rows, int64_t cols_pad, int64_t ld, int64_t cblk_pad, int64_t cblk_real,
                 float *out, int32_t accumulate, float *ws, void *stream) {
    if (!X || !out || !ws || cblk_pad < 1) return U2GNN_E_ARG;
    if (cols_pad == 0) return U2GNN_OK;
    int64_t chunks = (rows + CS_ROWS - 1) / CS_ROWS;
    hipStream_t st = u2gnn_stream(stream);
    const bool vec = al16(X) && al16(ws) && (ld & 3) == 0 && (cols_pad & 3) == 0;
    if (vec && rows <= SMALL_ROWS) {
        hipLaunchKernelGGL(colsum_small_kernel, dim3((unsigned)((cols_pad + 63) / 64)), dim3(1024), 0, st, X, rows,
                           cols_pad, ld, cblk_pad, cblk_real, out, accumulate);
        return u2gnn_launch_status();
    }
    const int rep = vec ? (int)std::max<int64_t>(1, (chunks + COLSUM_MAX_CHUNKS - 1) / COLSUM_MAX_CHUNKS) : 1;
    chunks = (chunks + rep - 1) / rep;   // never more than the CS_ROWS-row group count callers size ws by
    const unsigned nch = (unsigned)(chunks > 0 ? chunks : 1);
    if (vec)
        hipLaunchKernelGGL(rep > 1 ? colsum_partial_kernel<true> : colsum_partial_kernel<false>,
                           dim3((unsigned)((cols_pad + 255) / 256), nch), dim3(256), 0, st, X, rows, cols_pad, ld, rep, ws);
    else
        hipLaunchKernelGGL(colsum_partial_scalar_kernel, dim3((unsigned)((cols_pad + 63) / 64), nch), dim3(256), 0, st,
                           X, rows, cols_pad, ld, ws);
    hipLaunchKernelGGL(colsum_final_kernel, dim3((unsigned)((cols_pad + FIN_COLS - 1) / FIN_COLS)), dim3(256), 0, st, ws,
                       chunks > 0 ? chunks : 1, cols_pad, cblk_pad, cblk_real, out, accumulate);
    return u2gnn_launch_status();
}

int u2gnn_attn_softmax_fwd(const float *S, int64_t lds, float *P, float *Pd, int64_t ldp, int64_t rows_valid,
                           int64_t rows_pad, int64_t n_valid, int64_t n_pad, float p, uint64_t seed, uint32_t *keep,
                           int64_t ld_keep, void *stream) {
    if (!S || !Pd || (n_pad & 3) || (lds & 3) || (ldp & 3) || n_valid > n_pad || n_valid < 1) return U2GNN_E_ARG;
    if (Pd == P && p > 0.f) return U2GNN_E_ARG;
    if (!P && keep) return U2GNN_E_ARG;   // signed image: the sign bit is the keep bit
    if (keep && ((n_pad & 31) || ld_keep < n_pad / 32)) return U2GNN_E_ARG;
    if (n_pad > 1024 * SM_RV_MAX) return U2GNN_E_SHAPE;   // rows are held in registers
    hipStream_t st = u2gnn_stream(stream);
    // registers sized to the row (ceil(n_pad / 1024) float4 per thread up to 8): a fixed 8 made every
    // C4 row (4864 keys) compute 8192 exponentials, 3328 of them exp(-inf) = 0; the terms it drops are
    // exact zeros appended after the live ones, so P is bit-identical
    const int64_t rv = (n_pad + 1023) / 1024;
#define U2GNN_SMX(V) hipLaunchKernelGGL(attn_softmax_kernel<V>, dim3((unsigned)rows_pad), dim3(256), 0, st, S, lds, P, Pd, \
                                        ldp, rows_valid, n_valid, n_pad, p, seed, u2gnn_cur_epoch(), keep, ld_keep)
    if (rv <= 8) {
        switch (rv) {
            case 1: U2GNN_SMX(1); break;
            case 2: U2GNN_SMX(2); break;
            case 3: U2GNN_SMX(3); break;
            case 4: U2GNN_SMX(4); break;
            case 5: U2GNN_SMX(5); break;
            case 6: U2GNN_SMX(6); break;
            case 7: U2GNN_SMX(7); break;
            default: U2GNN_SMX(8); break;
        }
    }
#undef U2GNN_SMX
    else if (n_pad <= 16384)
        hipLaunchKernelGGL(attn_softmax_kernel<16>, dim3((unsigned)rows_pad), dim3(256), 0, st, S, lds, P, Pd, ldp,
                           rows_valid, n_valid, n_pad, p, seed, u2gnn_cur_epoch(), keep, ld_keep);
    else
        hipLaunchKernelGGL(attn_softmax_kernel<32>, dim3((unsigned)rows_pad), dim3(256), 0, st, S, lds, P, Pd, ldp,
                           rows_valid, n_valid, n_pad, p, seed, u2gnn_cur_epoch(), keep, ld_keep);
    return u2gnn_launch_status();
}

int u2gnn_split_x2(const float *src, int64_t ld_src, void *dst2, int64_t ld_dst2, int64_t rows, int64_t cols,
                   void *stream) {
    if (!src || !dst2 || rows < 0 || cols < 0 || (cols & 7) || (ld_src & 3) || (ld_dst2 & 15)) return U2GNN_E_ARG;
    if (!al16(src) || !al16(dst2)) return U2GNN_E_ALIGN;
    if (rows == 0 || cols == 0) return U2GNN_OK;
    const int64_t n = rows * (cols / 4);
    hipLaunchKernelGGL(split_x2_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, u2gnn_stream(stream), src,
                       ld_src, static_cast<__bf16 *>(dst2), ld_dst2, rows, cols);
    return u2gnn_launch_status();
}

int u2gnn_rowdot(const float *A, int64_t lda, const float *B, int64_t ldb, float *out, int64_t rows, int64_t cols,
                 void *stream) {
    if (!A || !B || !out) return U2GNN_E_ARG;
    if (rows == 0) return U2GNN_OK;
    hipLaunchKernelGGL(rowdot_kernel, dim3(grid_for(rows, 4, 1 << 30)), dim3(256), 0, u2gnn_stream(stream), A, lda, B,
                       ldb, out, rows, cols);
    return u2gnn_launch_status();
}

int u2gnn_layernorm_fwd(const float *Z, int64_t ldz, const float *gamma, const float *beta, float *Y, int64_t ldy,
                        float *mean, float *rstd, int64_t rows_valid, int64_t rows_pad, int64_t d, int64_t d_pad,
                        float eps, void *stream) {
    if (!Z || !gamma || !beta || !Y || !mean || !rstd || d < 1 || d > d_pad || d_pad > LN_MAXV * 64)
        return U2GNN_E_ARG;
    if (!al16(Z) || !al16(Y) || (ldz & 3) || (ldy & 3) || (d_pad & 3)) return U2GNN_E_ALIGN;
    // registers sized to the row: V4 = ceil(d_pad / 128) float4 per lane (C4: 3), not the maximum 8
    // (measured: the 8-wide arrays held ~160 VGPRs and 3 waves per SIMD for every width)
    hipStream_t st = u2gnn_stream(stream);
    const dim3 gr(grid_for(rows_pad, 8, 1 << 30));
#define U2GNN_LNF(V) hipLaunchKernelGGL((layernorm_fwd_kernel<V, 32>), gr, dim3(256), 0, st, Z, ldz, gamma, beta, Y, \
                                        ldy, mean, rstd, rows_valid, rows_pad, d, d_pad, eps)
    const int64_t v4 = (d_pad + 127) / 128;
    if (v4 <= 1) U2GNN_LNF(1);
    else if (v4 == 2) U2GNN_LNF(2);
    else if (v4 == 3) U2GNN_LNF(3);
    else if (v4 == 4) U2GNN_LNF(4);
    else U2GNN_LNF(LN_V4_MAX);
#undef U2GNN_LNF
    return u2gnn_launch_status();
}

namespace {
int layernorm_bwd_launch(const float *dY, int64_t ldy, const float *Z, int64_t ldz, const float *mean,
                         const float *rstd, const float *gamma, float *dZ, int64_t lddz, float *dZdrop, int64_t lddrop,
                         float p, uint64_t seed, int64_t rows_valid, int64_t rows_pad, int64_t d, int64_t d_pad,
                         const LnDelta *dt, void *stream) {
    if (!dY || !Z || !mean || !rstd || !gamma || !dZ || d < 1 || d > d_pad || d_pad > LN_MAXV * 64)
        return U2GNN_E_ARG;
    if (dt && dt->slabs && (dt->n_slab < 1 || !al16(dt->slabs) || (dt->slab_stride & 3))) return U2GNN_E_ARG;
    if (!al16(dY) || !al16(Z) || !al16(dZ) || (ldy & 3) || (ldz & 3) || (lddz & 3) || (d_pad & 3) ||
        (dZdrop && (!al16(dZdrop) || (lddrop & 3))))
        return U2GNN_E_ALIGN;
    if (dt && (!dt->X || !dt->bias || !dt->delta)) return U2GNN_E_ARG;
    if (dt && (!al16(dt->X) || !al16(dt->bias) || (dt->ldx & 3))) return U2GNN_E_ALIGN;
    const dim3 gr(grid_for(rows_pad, 8, 1 << 30));
    hipStream_t st = u2gnn_stream(stream);
    const LnDelta none{nullptr, 0, nullptr, nullptr, nullptr, 0, 0};
#define U2GNN_LNB(V)                                                                                                   \
    do {                                                                                                               \
        if (dt && dt->slabs)                                                                                           \
            hipLaunchKernelGGL((layernorm_bwd_kernel<V, true, true>), gr, dim3(256), 0, st, dY, ldy, Z, ldz, mean,    \
                               rstd, gamma, dZ, lddz, dZdrop, lddrop, p, seed, u2gnn_cur_epoch(), rows_valid, rows_pad, d, \
                               d_pad, *dt);                                                                            \
        else if (dt)                                                                                                   \
            hipLaunchKernelGGL((layernorm_bwd_kernel<V, true>), gr, dim3(256), 0, st, dY, ldy, Z, ldz, mean, rstd,    \
                               gamma, dZ, lddz, dZdrop, lddrop, p, seed, u2gnn_cur_epoch(), rows_valid, rows_pad, d,       \
                               d_pad, *dt);                                                                            \
        else                                                                                                           \
            hipLaunchKernelGGL((layernorm_bwd_kernel<V, false>), gr, dim3(256), 0, st, dY, ldy, Z, ldz, mean, rstd,   \
                               gamma, dZ, lddz, dZdrop, lddrop, p, seed, u2gnn_cur_epoch(), rows_valid, rows_pad, d,       \
                               d_pad, none);                                                                           \
    } while (0)
    const int64_t v4 = (d_pad + 127) / 128;
    if (v4 <= 1) U2GNN_LNB(1);
    else if (v4 == 2) U2GNN_LNB(2);
    else if (v4 == 3) U2GNN_LNB(3);
    else if (v4 == 4) U2GNN_LNB(4);
    else U2GNN_LNB(LN_V4_MAX);
#undef U2GNN_LNB
    return u2gnn_launch_status();
}
}  // namespace

int u2gnn_layernorm_bwd(const float *dY, int64_t ldy, const float *Z, int64_t ldz, const float *mean,
                        const float *rstd, const float *gamma, float *dZ, int64_t lddz, float *dZdrop, int64_t lddrop,
                        float p, uint64_t seed, int64_t rows_valid, int64_t rows_pad, int64_t d, int64_t d_pad,
                        void *stream) {
    return layernorm_bwd_launch(dY, ldy, Z, ldz, mean, rstd, gamma, dZ, lddz, dZdrop, lddrop, p, seed, rows_valid,
                                rows_pad, d, d_pad, nullptr, stream);
}

int u2gnn_layernorm_bwd_delta(const float *dY, int64_t ldy, const float *Z, int64_t ldz, const float *mean,
                              const float *rstd, const float *gamma, float *dZ, int64_t lddz, float *dZdrop,
                              int64_t lddrop, float p, uint64_t seed, int64_t rows_valid, int64_t rows_pad, int64_t d,
                              int64_t d_pad, const float *X, int64_t ldx, const float *bias, float *delta,
                              void *stream) {
    const LnDelta dt{X, ldx, bias, delta, nullptr, 0, 0};
    return layernorm_bwd_launch(dY, ldy, Z, ldz, mean, rstd, gamma, dZ, lddz, dZdrop, lddrop, p, seed, rows_valid,
                                rows_pad, d, d_pad, &dt, stream);
}

int u2gnn_layernorm_bwd_delta_slabs(float *dY, int64_t ldy, const float *slabs, int32_t n_slab, int64_t slab_stride,
                                    const float *Z, int64_t ldz, const float *mean, const float *rstd,
                                    const float *gamma, float *dZ, int64_t lddz, float *dZdrop, int64_t lddrop, float p,
                                    uint64_t seed, int64_t rows_valid, int64_t rows_pad, int64_t d, int64_t d_pad,
                                    const float *X, int64_t ldx, const float *bias, float *delta, void *stream) {
    if (!slabs) return U2GNN_E_ARG;
    const LnDelta dt{X, ldx, bias, delta, slabs, slab_stride, (int)n_slab};
    return layernorm_bwd_launch(dY, ldy, Z, ldz, mean, rstd, gamma, dZ, lddz, dZdrop, lddrop, p, seed, rows_valid,
                                rows_pad, d, d_pad, &dt, stream);
}

int u2gnn_layernorm_bwd_params(const float *dY, int64_t ldy, const float *Z, int64_t ldz, const float *mean,
                               const float *rstd, const float *dZdrop, int64_t lddrop, int64_t rows_valid, int64_t d,
                               int64_t d_pad, float *ws, float *dgamma, float *dbeta, float *dbias, void *stream) {
    if (!dY || !Z || !mean || !rstd || !ws || !dgamma || !dbeta || d < 1 || d > d_pad) return U2GNN_E_ARG;
    if (dbias && !dZdrop) return U2GNN_E_ARG;
    if (!al16(dY) || !al16(Z) || !al16(ws) || (ldy & 3) || (ldz & 3) || (d_pad & 3) ||
        (dbias && (!al16(dZdrop) || (lddrop & 3))))
        return U2GNN_E_ALIGN;
    const int64_t groups = rows_valid > 0 ? (rows_valid + CS_ROWS - 1) / CS_ROWS : 1;
    const int rep = (int)((groups + LN_MAX_CHUNKS - 1) / LN_MAX_CHUNKS);
    const int64_t chunks = (groups + rep - 1) / rep;   // <= the CS_ROWS-row group count callers size ws by
    hipStream_t st = u2gnn_stream(stream);
    if (rows_valid <= SMALL_ROWS) {
        hipLaunchKernelGGL(ln_params_small_kernel, dim3((unsigned)((d_pad + 63) / 64)), dim3(1024), 0, st, dY, ldy, Z,
                           ldz, mean, rstd, dbias ? dZdrop : nullptr, lddrop, rows_valid, d, d_pad, dgamma, dbeta,
                           dbias);
        return u2gnn_launch_status();
    }
    hipLaunchKernelGGL(rep > 1 ? ln_colstats_kernel<true> : ln_colstats_kernel<false>,
                       dim3((unsigned)((d_pad + 255) / 256), (unsigned)chunks), dim3(256), 0, st, dY,
                       ldy, Z, ldz, mean, rstd, dbias ? dZdrop : nullptr, lddrop, rows_valid, d, d_pad, rep, ws);
    hipLaunchKernelGGL(ln_param_reduce_kernel, dim3((unsigned)((d + FIN_COLS - 1) / FIN_COLS)), dim3(256), 0, st, ws,
                       chunks, d, d_pad,
                       dgamma, dbeta, dbias);
    return u2gnn_launch_status();
}

}  // extern "C"

namespace {

// the launch geometry of one public job, exactly as its single-job entry point chooses it
struct RbPlan {
    bool small;            // one-launch small form (1024 threads)
    int64_t chunks;        // partial rows (COLSUM / LNPARAMS, long form)
    int rep;               // fold factor of the partial pass
    int64_t ws_floats;     // partial sums (long form)
};

// ptrs = false: shapes only (the layer executor sizes its workspace before any buffer exists)
int rb_plan(const u2gnn_reduce_job &J, RbPlan &p, bool ptrs = true) {
    p = RbPlan{false, 0, 1, 0};
    switch (J.kind) {
        case U2GNN_RJOB_SLAB:
            if (J.n_slab < 1 || J.rblk_pad < 1 || J.cblk_pad < 1 || J.rows < 0 || J.cols < 0) return U2GNN_E_ARG;
            if (!ptrs) return U2GNN_OK;
            if (!J.src || !J.dst) return U2GNN_E_ARG;
            if (!al16(J.src) || (J.cols & 3) || (J.ld_src & 3) || (J.slab_stride & 3)) return U2GNN_E_ALIGN;
            return U2GNN_OK;
        case U2GNN_RJOB_COLSUM: {   // u2gnn_colsum, vectorised forms only
            if (J.cblk_pad < 1 || J.rows < 0 || J.cols < 0) return U2GNN_E_ARG;
            if (ptrs && (!J.src || !J.dst)) return U2GNN_E_ARG;
            if ((ptrs && !al16(J.src)) || (J.ld_src & 3) || (J.cols & 3)) return U2GNN_E_ALIGN;
            p.small = J.rows <= SMALL_ROWS;
            int64_t chunks = (J.rows + CS_ROWS - 1) / CS_ROWS;
            p.rep = (int)std::max<int64_t>(1, (chunks + COLSUM_MAX_CHUNKS - 1) / COLSUM_MAX_CHUNKS);
            chunks = (chunks + p.rep - 1) / p.rep;
            p.chunks = chunks > 0 ? chunks : 1;
            if (!p.small) p.ws_floats = (p.chunks * J.cols + 3) / 4 * 4;
            return U2GNN_OK;
        }
        case U2GNN_RJOB_LNPARAMS: {   // u2gnn_layernorm_bwd_params
            if (J.d < 1 || J.d > J.cols) return U2GNN_E_ARG;
            if (ptrs) {
                if (!J.src || !J.Z || !J.mean || !J.rstd || !J.dst || !J.dbeta) return U2GNN_E_ARG;
                if (J.dbias && !J.dZdrop) return U2GNN_E_ARG;
                if (!al16(J.src) || !al16(J.Z) || (J.dbias && !al16(J.dZdrop))) return U2GNN_E_ALIGN;
            }
            if ((J.ld_src & 3) || (J.ldz & 3) || (J.cols & 3) || (J.dbias && (J.lddrop & 3))) return U2GNN_E_ALIGN;
            p.small = J.rows <= SMALL_ROWS;
            const int64_t groups = J.rows > 0 ? (J.rows + CS_ROWS - 1) / CS_ROWS : 1;
            p.rep = (int)((groups + LN_MAX_CHUNKS - 1) / LN_MAX_CHUNKS);
            p.chunks = (groups + p.rep - 1) / p.rep;
            if (!p.small) p.ws_floats = p.chunks * 3 * J.cols;
            return U2GNN_OK;
        }
        default: return U2GNN_E_ARG;
    }
}

template <int NT>
int rb_launch(std::vector<RbJob> &jobs, hipStream_t st) {
    for (size_t o = 0; o < jobs.size(); o += RB_MAX) {
        RbBatch B;
        std::memset(&B, 0, sizeof(B));
        B.n = (int32_t)std::min<size_t>(RB_MAX, jobs.size() - o);
        int64_t blocks = 0;
        for (int i = 0; i < B.n; ++i) B.j[i] = jobs[o + i], blocks += B.j[i].nblk;
        if (blocks <= 0) continue;
        if (blocks >= (int64_t)1 << 31) return U2GNN_E_SHAPE;
        hipLaunchKernelGGL(reduce_batch_kernel<NT>, dim3((unsigned)blocks), dim3(NT), 0, st, B);
    }
    return u2gnn_launch_status();
}

}  // namespace

extern "C" {

int u2gnn_slab_bias_drop_resid_ln(const float *src, int32_t n_slab, int64_t slab_stride, int64_t ld_src,
                                   const float *bias, const float *resid, int64_t ld_res, float p, uint64_t seed,
                                   float *Z, int64_t ldz, const float *gamma, const float *beta, float *Y, int64_t ldy,
                                   float *mean, float *rstd, int64_t d, int64_t rows_valid, int64_t rows_pad, float eps,
                                   void *stream) {
    const int64_t dp = (d + 63) / 64 * 64;   // padded width: columns per lane = dp / 64
    if (!src || !bias || !resid || !Z || !gamma || !beta || !Y || !mean || !rstd || n_slab < 1 || d < 1 || d > 256 ||
        rows_valid > rows_pad || ld_src < dp || ld_res < dp || ldz < dp || ldy < dp || p < 0.f || p >= 1.f)
        return U2GNN_E_ARG;
    if (rows_pad <= 0) return U2GNN_OK;
    const dim3 grid((unsigned)((rows_pad + 3) / 4));
    hipStream_t st = u2gnn_stream(stream);
#define U2GNN_SLAB_LN(CPL)                                                                                       \
    hipLaunchKernelGGL(slab_bias_drop_resid_ln_kernel<CPL>, grid, dim3(256), 0, st, src, n_slab, slab_stride, ld_src, \
                       bias, resid, ld_res, p, seed, u2gnn_cur_epoch(), Z, ldz, gamma, beta, Y, ldy, mean, rstd, d,      \
                       rows_valid, rows_pad, eps)
    switch (dp / 64) {
        case 1: U2GNN_SLAB_LN(1); break;
        case 2: U2GNN_SLAB_LN(2); break;
        case 3: U2GNN_SLAB_LN(3); break;
        default: U2GNN_SLAB_LN(4); break;
    }
#undef U2GNN_SLAB_LN
    return u2gnn_launch_status();
}

int64_t u2gnn_reduce_batch_ws_floats(const u2gnn_reduce_job *jobs, int32_t n) {
    if (n < 0 || (n && !jobs)) return -1;
    int64_t tot = 0;
    for (int32_t i = 0; i < n; ++i) {
        RbPlan p;
        if (rb_plan(jobs[i], p, false) != U2GNN_OK) return -1;
        tot += p.ws_floats;
    }
    return tot;
}

int u2gnn_reduce_batch(const u2gnn_reduce_job *jobs, int32_t n, float *ws, int64_t ws_floats, void *stream) {
    if (n < 0 || (n && !jobs)) return U2GNN_E_ARG;
    if (ws && !al16(ws)) return U2GNN_E_ALIGN;
    std::vector<RbJob> part, fin, small, zero;
    std::vector<const u2gnn_reduce_job *> slabs;
    int64_t off = 0;
    for (int32_t i = 0; i < n; ++i) {
        const u2gnn_reduce_job &J = jobs[i];
        RbPlan p;
        const int rc = rb_plan(J, p);
        if (rc != U2GNN_OK) return rc;
        if (J.kind == U2GNN_RJOB_SLAB) {
            if (J.rows > 0 && J.cols > 0) slabs.push_back(&J);
            continue;
        }
        RbJob r;
        std::memset(&r, 0, sizeof(r));
        r.src = J.src, r.ld_src = J.ld_src, r.rows = J.rows, r.cols = J.cols, r.flag = J.accumulate;
        r.cbp = J.cblk_pad, r.cbr = J.cblk_real, r.o0 = J.dst;
        const bool ln = J.kind == U2GNN_RJOB_LNPARAMS;
        if (ln) {
            r.Z = J.Z, r.ldz = J.ldz, r.mean = J.mean, r.rstd = J.rstd, r.dZd = J.dbias ? J.dZdrop : nullptr;
            r.lddrop = J.lddrop, r.d = J.d, r.o1 = J.dbeta, r.o2 = J.dbias;
        } else if (J.cols == 0) {
            continue;   // u2gnn_colsum: nothing to sum
        }
        if (!ln && J.rows == 0) {   // an all-zero column sum (the in-projection's key bias: encoder_layer.cpp)
            zero.push_back(r);
            continue;
        }
        if (p.small) {
            r.kind = ln ? RB_LN_SMALL : RB_CS_SMALL;
            r.nblk = (int32_t)((J.cols + 63) / 64);
            small.push_back(r);
            continue;
        }
        if (!ws || off + p.ws_floats > ws_floats) return U2GNN_E_ARG;
        r.ws = ws + off;
        off += p.ws_floats;
        RbJob q = r;
        q.kind = ln ? RB_LN_PART : RB_CS_PART;
        q.nbx = (int32_t)((J.cols + 255) / 256);
        q.nblk = q.nbx * (int32_t)p.chunks;
        q.n = p.rep;
        part.push_back(q);
        r.kind = ln ? RB_LN_FINAL : RB_CS_FINAL;
        r.nblk = (int32_t)(((ln ? J.d : J.cols) + FIN_COLS - 1) / FIN_COLS);
        r.n = (int32_t)p.chunks;
        fin.push_back(r);
    }
    // An all-zero column sum rides with a launch that runs anyway: the single-pass small jobs' when there are
    // any (C2, C3: every column sum is small, so no final pass is launched for it), else the final pass over
    // no partials (C5: the slab reductions then need no 1024-thread launch of their own) -- same zeros either way
    for (RbJob &r : zero) {
        if (!small.empty()) {
            r.kind = RB_CS_SMALL;
            r.nblk = (int32_t)((r.cols + 63) / 64);
            small.push_back(r);
        } else {
            r.kind = RB_CS_FINAL;
            r.nblk = (int32_t)((r.cols + FIN_COLS - 1) / FIN_COLS);
            r.n = 0;
            fin.push_back(r);
        }
    }
    // slab jobs ride with the small jobs' launch when there is one (per-thread bodies: any block size)
    const int slab_nt = small.empty() ? 256 : 1024;
    for (const u2gnn_reduce_job *J : slabs) {
        RbJob r;
        std::memset(&r, 0, sizeof(r));
        r.kind = RB_SLAB;
        r.src = J->src, r.n = J->n_slab, r.stride = J->slab_stride, r.rows = J->rows, r.cols = J->cols;
        r.ld_src = J->ld_src, r.rbp = J->rblk_pad, r.rbr = J->rblk_real, r.cbp = J->cblk_pad, r.cbr = J->cblk_real;
        r.o0 = J->dst, r.ld_dst = J->ld_dst, r.alpha = J->alpha, r.flag = J->accumulate;
        r.vec = J->cblk_pad == J->cblk_real && al16(J->dst) && (J->ld_dst & 3) == 0;
        const int64_t nb = (J->rows * (J->cols / 4) + slab_nt - 1) / slab_nt;
        if (nb >= (int64_t)1 << 31) return U2GNN_E_SHAPE;
        r.nblk = (int32_t)nb;
        (small.empty() ? fin : small).push_back(r);
    }
    hipStream_t st = u2gnn_stream(stream);
    int rc = rb_launch<256>(part, st);
    if (rc == U2GNN_OK) rc = rb_launch<256>(fin, st);
    if (rc == U2GNN_OK) rc = rb_launch<1024>(small, st);
    return rc;
}

int u2gnn_dropout(const float *X, int64_t ldx, float *Y, int64_t ldy, int64_t rows, int64_t cols, float p,
                  uint64_t seed, void *stream) {
    if (!X || !Y || p < 0.f || p >= 1.f) return U2GNN_E_ARG;
    if (rows * cols == 0) return U2GNN_OK;
    hipLaunchKernelGGL(dropout_kernel, dim3(grid_for(rows * cols, 256)), dim3(256), 0, u2gnn_stream(stream), X, ldx, Y,
                       ldy, rows, cols, p, seed, u2gnn_cur_epoch());
    return u2gnn_launch_status();
}

int u2gnn_dropout_mask(uint64_t seed, int64_t rows, int64_t cols, float p, uint8_t *out, void *stream) {
    if (!out) return U2GNN_E_ARG;
    hipLaunchKernelGGL(dropout_mask_kernel, dim3(grid_for(rows * cols, 256)), dim3(256), 0, u2gnn_stream(stream), seed, u2gnn_cur_epoch(),
                       rows, cols, p, out);
    return u2gnn_launch_status();
}

}  // extern "C"
