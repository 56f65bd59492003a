/*
 * u2gnn_lus.h — C ABI of libu2gnn_lus.so, the host-side natives: the log-uniform sampler used by
 * the sampled-softmax loss, and the batch assembler (end of file).  Replaces the reference's C++ class + Cython binding:
 *   Log_Uniform_Sampler.h:9-24 / Log_Uniform_Sampler.cpp:10-88 and log_uniform.pyx:16-40
 *   (U2GNN_pytorch/log_uniform/), called from sampled_softmax.py:31.
 * Same engine (std::default_random_engine = minstd_rand0, seed 1111 by default), same
 * uniform_real_distribution<double>, same lround(exp(x*log N)) - 1 map and the same
 * std::unordered_set<long> insertion sequence, so sample sets AND their iteration order
 * equal the reference's for the same libstdc++.
 * No C++ exception crosses the ABI; errors are int status codes:
 *   0 ok, -1 bad argument (null handle, size > N: the reference would loop forever),
 *   -2 allocation failure.
 * Threading: a handle owns a mutable engine; calls on one handle must be serialised
 * (the reference calls it once per training step on the training thread).
 */
#ifndef U2GNN_LUS_H
#define U2GNN_LUS_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* LogUniformSampler(N)  (log_uniform.pyx:19-20; Log_Uniform_Sampler.cpp:10-16) */
void *u2gnn_lus_create(int64_t range_max, uint32_t seed);
void u2gnn_lus_destroy(void *h);
/* sample(size) (Log_Uniform_Sampler.cpp:57-71): `size` distinct ids in unordered_set order. */
int u2gnn_lus_sample(void *h, size_t size, int64_t *out_ids, int32_t *num_tries);
/* sample(size) as the reference's Python binding returns it (log_uniform.pyx:24-27 converts the unordered_set
 * into a Python set, then list()): the same ids in CPython set order -- list(set(u2gnn_lus_sample's ids)) without
 * the interpreter round trip (round 6: that conversion was about half of the per-step sampler time). */
int u2gnn_lus_sample_pyset(void *h, size_t size, int64_t *out_ids, int32_t *num_tries);
/* expected_count (Log_Uniform_Sampler.cpp:23-32) */
int u2gnn_lus_expected_count(void *h, int32_t num_tries, const int64_t *ids, size_t n, float *out);
/* probability (Log_Uniform_Sampler.cpp:18-21) */
float u2gnn_lus_probability(void *h, int64_t idx);
/* sample_unique (Log_Uniform_Sampler.cpp:73-88): ids not in `excluded`; rejects size > N - |excluded| */
int u2gnn_lus_sample_unique(void *h, size_t size, const int64_t *excluded, size_t n_excluded, int64_t *out_ids);
/* accidental_matches (Log_Uniform_Sampler.cpp:34-55): pairs (label index, sample index),
 * written to out_pairs[2*k], out_pairs[2*k+1]; *n_out = number of pairs; capacity in pairs. */
int u2gnn_lus_accidental_matches(const int64_t *labels, size_t n_labels, const int64_t *samples,
                                 size_t n_samples, int64_t *out_pairs, size_t capacity, size_t *n_out);

/* ---- host batch assembly (csrc/batch_assembly.cpp) -----------------------------------
 * get_batch_data / Batch_Loader (train_pytorch_U2GNN_Sup.py:99-126, train_pytorch_U2GNN_UnSup.py:
 * 101-134) for the graphs `ids` (a permutation prefix drawn by the caller): offsets [n_ids+1],
 * input_x [N, k+1] (row i: i, then k neighbours drawn with replacement, as batch rows; isolated
 * nodes repeat i) and gnode [N] (dataset-global node id of each row).  The neighbour draws continue
 * numpy's legacy MT19937 global stream given as (mt_key[624], *mt_pos) from np.random.get_state()
 * exactly as np.random.randint(0, deg[:, None], size=(n, k)) over the non-isolated nodes does
 * (masked rejection on 32-bit outputs); the advanced state is written back in place.  Graph g owns
 * global nodes node_start[g] .. +n_nodes[g]; node v's neighbours (ids local to its graph, in the
 * reference's edge order) are nbr[nbr_start[v] .. + deg[v]].  n_cap: rows available in input_x /
 * gnode.  Returns 0, or -1 for a bad argument / N > n_cap. */
int u2gnn_batch_assemble(uint32_t *mt_key, int32_t *mt_pos, const int64_t *ids, int64_t n_ids,
                         const int64_t *n_nodes, const int64_t *node_start, const int64_t *deg,
                         const int64_t *nbr_start, const int64_t *nbr, int32_t k, int64_t n_cap,
                         int64_t *offsets, int64_t *input_x, int64_t *gnode);

#ifdef __cplusplus
}
#endif
#endif
