// Cost of the split-K "last block reduces" handshake on gfx950: every block stores its slab tile
// (BM x BN fp32), counts itself in on the tile's agent-scope counter, and the last-arriving block
// sums the tile's slabs.  Variants: FENCE = device-scope release/acquire fences around the counter
// (the C++ model's way); COHERENT = slab stores and the last block's loads carry the agent-scope
// coherence bit (the code the compiler emits for relaxed agent-scope atomic stores / loads) and the
// counter increment waits for the stores to complete, no cache-wide fence.  Compared with the same
// stores plus a separate reduce launch.  Build: hipcc --offload-arch=gfx950 -O3 tools/micro/fence_bench.hip -o /tmp/fb
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f4v __attribute__((ext_vector_type(4)));
constexpr int kCoherent = 16;   // cache-policy aux bit of the agent-scope coherent accesses

template <int MODE>   // 0 stores only, 1 fenced handshake, 2 coherent-access handshake
__global__ void __launch_bounds__(256) slab_kernel(float *slabs, float *out, int *cnt, int tiles, int split,
                                                   int tile_elems) {
    const int tile = blockIdx.x % tiles, z = blockIdx.x / tiles;
    float *s = slabs + ((size_t)z * tiles + tile) * tile_elems;
    if constexpr (MODE == 2) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(s, 0, 0x7fffffff, 0x00020000);
        for (int i = threadIdx.x * 4; i < tile_elems; i += 1024) {
            const f4v v = {z + 1.f, (float)z, (float)i, (float)tile};
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v),
                                                   rs, i * 4, 0, kCoherent);
        }
        __shared__ int last2;
        __builtin_amdgcn_s_waitcnt(0);   // this thread's slab stores have completed
        __syncthreads();
        if (threadIdx.x == 0) last2 = __hip_atomic_fetch_add(cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == split - 1;
        __syncthreads();
        if (!last2) return;
        for (int i = threadIdx.x * 4; i < tile_elems; i += 1024) {
            float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
            for (int q = 0; q < split; ++q) {
                const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc(
                    slabs + ((size_t)q * tiles + tile) * tile_elems, 0, 0x7fffffff, 0x00020000);
                const auto u = __builtin_amdgcn_raw_buffer_load_b128(rq, i * 4, 0, kCoherent);
                const f4v v = __builtin_bit_cast(f4v, u);
                a.x += v.x, a.y += v.y, a.z += v.z, a.w += v.w;
            }
            *reinterpret_cast<float4 *>(out + (size_t)tile * tile_elems + i) = a;
        }
        if (threadIdx.x == 0) __hip_atomic_store(cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    for (int i = threadIdx.x * 4; i < tile_elems; i += 1024)
        *reinterpret_cast<float4 *>(s + i) = make_float4(z + 1.f, z, i, tile);
    if constexpr (MODE == 1) {
        __shared__ int last;
        __threadfence();
        __syncthreads();
        if (threadIdx.x == 0) last = atomicAdd(cnt + tile, 1) == split - 1;
        __syncthreads();
        if (!last) return;
        __threadfence();
        for (int i = threadIdx.x * 4; i < tile_elems; i += 1024) {
            float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
            for (int q = 0; q < split; ++q) {
                const float4 v = *reinterpret_cast<const float4 *>(slabs + ((size_t)q * tiles + tile) * tile_elems + i);
                a.x += v.x, a.y += v.y, a.z += v.z, a.w += v.w;
            }
            *reinterpret_cast<float4 *>(out + (size_t)tile * tile_elems + i) = a;
        }
        if (threadIdx.x == 0) atomicExch(cnt + tile, 0);
    }
}

__global__ void reduce_kernel(const float *slabs, float *out, int tiles, int split, int tile_elems) {
    const size_t n = (size_t)tiles * tile_elems;
    for (size_t i = ((size_t)blockIdx.x * 256 + threadIdx.x) * 4; i < n; i += (size_t)gridDim.x * 1024) {
        float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int q = 0; q < split; ++q) {
            const float4 v = *reinterpret_cast<const float4 *>(slabs + (size_t)q * n + i);
            a.x += v.x, a.y += v.y, a.z += v.z, a.w += v.w;
        }
        *reinterpret_cast<float4 *>(out + i) = a;
    }
}

int main() {
    struct Case { int tiles, split, tile_elems; const char *name; };
    const Case cases[] = {{30, 14, 64 * 64, "C5 P.V 64x64 x30 tiles, split 14"},
                          {6, 16, 64 * 64, "C5 wgrad 64x64 x6 tiles, split 16"},
                          {57, 4, 256 * 128, "C4 P.V 256x128 x57 tiles, split 4"}};
    float *slabs, *out;
    int *cnt;
    hipMalloc(&slabs, 64 << 20);
    hipMalloc(&out, 16 << 20);
    hipMalloc(&cnt, 4096 * 4);
    hipMemset(cnt, 0, 4096 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int reps = 200;
    for (const Case &c : cases) {
        const int blocks = c.tiles * c.split;
        float t[4];
        for (int mode = 0; mode < 4; ++mode) {
            for (int w = 0; w < 10; ++w) {
                if (mode == 0) slab_kernel<0><<<blocks, 256>>>(slabs, out, cnt, c.tiles, c.split, c.tile_elems);
                if (mode == 1) {
                    slab_kernel<0><<<blocks, 256>>>(slabs, out, cnt, c.tiles, c.split, c.tile_elems);
                    reduce_kernel<<<1024, 256>>>(slabs, out, c.tiles, c.split, c.tile_elems);
                }
                if (mode == 2) slab_kernel<1><<<blocks, 256>>>(slabs, out, cnt, c.tiles, c.split, c.tile_elems);
                if (mode == 3) slab_kernel<2><<<blocks, 256>>>(slabs, out, cnt, c.tiles, c.split, c.tile_elems);
            }
            hipEventRecord(e0);
            for (int r = 0; r < reps; ++r) {
                if (mode == 0) slab_kernel<0><<<blocks, 256>>>(slabs, out, cnt, c.tiles, c.split, c.tile_elems);
                if (mode == 1) {
                    slab_kernel<0><<<blocks, 256>>>(slabs, out, cnt, c.tiles, c.split, c.tile_elems);
                    reduce_kernel<<<1024, 256>>>(slabs, out, c.tiles, c.split, c.tile_elems);
                }
                if (mode == 2) slab_kernel<1><<<blocks, 256>>>(slabs, out, cnt, c.tiles, c.split, c.tile_elems);
                if (mode == 3) slab_kernel<2><<<blocks, 256>>>(slabs, out, cnt, c.tiles, c.split, c.tile_elems);
            }
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            hipEventElapsedTime(&t[mode], e0, e1);
        }
        // full check of the last (coherent) run: every element of every tile
        std::vector<float> h((size_t)c.tiles * c.tile_elems);
        hipMemcpy(h.data(), out, h.size() * 4, hipMemcpyDeviceToHost);
        size_t bad = 0;
        for (int tl = 0; tl < c.tiles; ++tl)
            for (int i = 0; i < c.tile_elems; ++i) {
                float w[4] = {0.f, 0.f, 0.f, 0.f};
                for (int z = 0; z < c.split; ++z) w[0] += z + 1.f, w[1] += z, w[2] += (float)(i & ~3), w[3] += tl;
                bad += h[(size_t)tl * c.tile_elems + i] != w[i & 3];
            }
        printf("%-40s stores %6.2f us | + reduce launch %6.2f | fenced %6.2f | coherent %6.2f us  (%zu bad)\n",
               c.name, 1e3f * t[0] / reps, 1e3f * t[1] / reps, 1e3f * t[2] / reps, 1e3f * t[3] / reps, bad);
    }
    return 0;
}
