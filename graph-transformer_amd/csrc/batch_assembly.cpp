// Native host batch assembly: get_batch_data / Batch_Loader of the reference
// (train_pytorch_U2GNN_Sup.py:99-126, train_pytorch_U2GNN_UnSup.py:101-134) for the graphs a
// permutation selected, bit-exact with the reference's per-node Python loop AND leaving numpy's
// global random stream in the state that loop leaves it.
//
// The reference draws, node by node, np.random.choice(nbrs, k, replace=True) from the legacy
// global RandomState (MT19937); u2gnn_hip/batching.py already replaces that loop by ONE
// np.random.randint(0, deg[live][:, None], size=(n_live, k)), which consumes the stream
// identically.  That call costs ~2 ms per 64-graph COLLAB batch on one core (numpy's broadcast
// path), more than a GPU training step, so this file continues the same MT19937 stream in C++:
//   * the caller passes numpy's state (key[624], pos) from np.random.get_state() and writes the
//     advanced state back with np.random.set_state();
//   * legacy RandomState.randint on int64 with per-element bounds (numpy
//     random/_bounded_integers _rand_int64 -> random_bounded_uint64, use_masked=True): for range
//     r = high - 1 - low, r == 0 draws nothing, otherwise masked rejection on 32-bit outputs:
//     v = next_uint32() & mask until v <= r, mask = 2^ceil(log2(r+1)) - 1;
//   * the draws are taken in C order over [n_live, k], i.e. node by node, k per node.
// No exceptions cross the ABI; int status codes as in u2gnn_lus.h.
#include <cstdint>
#include <cstring>

#include "u2gnn_lus.h"

namespace {

constexpr int MT_N = 624, MT_M = 397;

struct MT {
    uint32_t *key;
    int pos;
    void gen() {   // numpy mt19937_gen (the reference MT19937 twist)
        constexpr uint32_t UPPER = 0x80000000u, LOWER = 0x7fffffffu, MATA = 0x9908b0dfu;
        int i = 0;
        uint32_t y;
        for (; i < MT_N - MT_M; ++i) {
            y = (key[i] & UPPER) | (key[i + 1] & LOWER);
            key[i] = key[i + MT_M] ^ (y >> 1) ^ (-(y & 1u) & MATA);
        }
        for (; i < MT_N - 1; ++i) {
            y = (key[i] & UPPER) | (key[i + 1] & LOWER);
            key[i] = key[i + (MT_M - MT_N)] ^ (y >> 1) ^ (-(y & 1u) & MATA);
        }
        y = (key[MT_N - 1] & UPPER) | (key[0] & LOWER);
        key[MT_N - 1] = key[MT_M - 1] ^ (y >> 1) ^ (-(y & 1u) & MATA);
        pos = 0;
    }
    uint32_t next32() {   // numpy mt19937_next32
        if (pos == MT_N) gen();
        uint32_t y = key[pos++];
        y ^= (y >> 11);
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= (y >> 18);
        return y;
    }
};

inline uint32_t mask_for(uint32_t r) {
    r |= r >> 1;
    r |= r >> 2;
    r |= r >> 4;
    r |= r >> 8;
    r |= r >> 16;
    return r;
}

}  // namespace

extern "C" int u2gnn_batch_assemble(uint32_t *mt_key, int32_t *mt_pos, const int64_t *ids, int64_t n_ids,
                                    const int64_t *n_nodes, const int64_t *node_start, const int64_t *deg,
                                    const int64_t *nbr_start, const int64_t *nbr, int32_t k, int64_t n_cap,
                                    int64_t *offsets, int64_t *input_x, int64_t *gnode) {
    if (!mt_key || !mt_pos || (!ids && n_ids) || !n_nodes || !node_start || !deg || !nbr_start || !offsets ||
        n_ids < 0 || k < 0 || *mt_pos < 0 || *mt_pos > MT_N)
        return -1;
    offsets[0] = 0;
    for (int64_t b = 0; b < n_ids; ++b) offsets[b + 1] = offsets[b] + n_nodes[ids[b]];
    const int64_t N = offsets[n_ids];
    if (N > n_cap || (N && (!input_x || !gnode)) || (k && N && !nbr)) return -1;
    MT mt{mt_key, *mt_pos};
    const int64_t W = (int64_t)k + 1;
    for (int64_t b = 0; b < n_ids; ++b) {
        const int64_t g = ids[b], s0 = node_start[g], n = n_nodes[g], o = offsets[b];
        for (int64_t i = 0; i < n; ++i) {
            const int64_t node = s0 + i, row = o + i;
            int64_t *x = input_x + row * W;
            gnode[row] = node;
            x[0] = row;
            const int64_t dg = deg[node];
            if (dg <= 0) {   // isolated: [u] * (k+1), no draw
                for (int j = 1; j <= k; ++j) x[j] = row;
                continue;
            }
            const uint32_t r = (uint32_t)(dg - 1), m = mask_for(r);
            const int64_t *nb = nbr + nbr_start[node];
            for (int j = 1; j <= k; ++j) {
                uint32_t v = 0;
                if (r) {
                    do {
                        v = mt.next32() & m;
                    } while (v > r);
                }
                x[j] = nb[v] + o;   // neighbour id within its graph -> batch row
            }
        }
    }
    *mt_pos = mt.pos;
    return 0;
}
