// Host-side log-uniform sampler for the sampled-softmax loss (C ABI: include/u2gnn_lus.h).
// A new implementation of the reference's sampler contract (see the header for citations);
// it keeps the reference's engine and set semantics so the drawn ids are identical.
#include "u2gnn_lus.h"

#include <cmath>
#include <cstdlib>
#include <functional>
#include <new>
#include <random>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace {
// Bump allocator for one draw's unordered_set (nodes and bucket arrays; freeing is a no-op, the arena is
// rewound per call).  The set's iteration order depends only on its hash policy and insertion sequence,
// never on the allocator, so the ids and their order are unchanged; what goes is a malloc / free per try
// (emplace builds the node before it finds a duplicate).  Blocks are kept across calls.
struct Arena {
    std::vector<char *> blocks;
    size_t blk = 0, off = 0;
    static constexpr size_t BLOCK = 1 << 20;
    void *get(size_t bytes, size_t align) {
        if (bytes > BLOCK) throw std::bad_alloc();
        off = (off + align - 1) & ~(align - 1);
        if (blocks.empty() || off + bytes > BLOCK) {
            if (!blocks.empty()) ++blk;
            if (blk == blocks.size()) {
                char *b = static_cast<char *>(std::malloc(BLOCK));
                if (!b) throw std::bad_alloc();
                blocks.push_back(b);
            }
            off = 0;
        }
        void *p = blocks[blk] + off;
        off += bytes;
        return p;
    }
    void rewind() { blk = 0, off = 0; }
    ~Arena() {
        for (char *b : blocks) std::free(b);
    }
};

template <class T>
struct ArenaAlloc {
    using value_type = T;
    Arena *a;
    explicit ArenaAlloc(Arena *a_) : a(a_) {}
    template <class U>
    ArenaAlloc(const ArenaAlloc<U> &o) : a(o.a) {}
    T *allocate(size_t n) { return static_cast<T *>(a->get(n * sizeof(T), alignof(T))); }
    void deallocate(T *, size_t) {}
    template <class U>
    bool operator==(const ArenaAlloc<U> &o) const { return a == o.a; }
    template <class U>
    bool operator!=(const ArenaAlloc<U> &o) const { return a != o.a; }
};
using IdSet = std::unordered_set<long, std::hash<long>, std::equal_to<long>, ArenaAlloc<long>>;

struct Sampler {
    int64_t n;
    std::minstd_rand0 engine;                    // == std::default_random_engine (libstdc++)
    std::uniform_real_distribution<double> uni;  // [0, 1)
    std::vector<float> prob;
    Arena arena;
    std::vector<int64_t> pytab;                  // sample_pyset's table
    Sampler(int64_t n_, uint32_t seed) : n(n_), engine(seed), uni(0.0, 1.0), prob((size_t)n_) {
        const double lr = std::log((double)(n_ + 1));
        for (int64_t i = 0; i < n_; ++i) prob[(size_t)i] = (float)((std::log((double)(i + 2)) - std::log((double)(i + 1))) / lr);
    }
    long draw(double log_n) { return std::lround(std::exp(uni(engine) * log_n)) - 1; }
};

// CPython's set of non-negative ints (Objects/setobject.c, 3.x: hash(i) = i, 8-slot start, 9 linear probes then
// perturbed probing, resize to 4 x used once fill * 5 >= mask * 3, rehash in table order): the order of
// list(set(ids)) for distinct ids inserted in the given order -- what the reference's Cython binding
// returns (a Python set built from the C++ unordered_set, then list()).  tests/test_sampler_cpu.py checks it
// against this interpreter's own set on thousands of draws.
struct PySetOrder {
    static constexpr int64_t EMPTY = -1;
    static constexpr size_t LINEAR_PROBES = 9, PERTURB_SHIFT = 5;
    std::vector<int64_t> &tab;
    size_t mask = 7, fill = 0;
    explicit PySetOrder(std::vector<int64_t> &t) : tab(t) { tab.assign(8, EMPTY); }
    static void put(std::vector<int64_t> &t, size_t mask, int64_t key) {
        size_t perturb = (size_t)key, i = (size_t)key & mask;
        while (true) {
            const size_t probes = i + LINEAR_PROBES <= mask ? LINEAR_PROBES : 0;
            for (size_t j = 0; j <= probes; ++j)
                if (t[i + j] == EMPTY) {
                    t[i + j] = key;
                    return;
                }
            perturb >>= PERTURB_SHIFT;
            i = (i * 5 + 1 + perturb) & mask;
        }
    }
    void add(int64_t key) {   // key not yet present
        put(tab, mask, key);
        ++fill;
        if (fill * 5 < mask * 3) return;
        const size_t minused = fill > 50000 ? fill * 2 : fill * 4;
        size_t newsize = 8;
        while (newsize <= minused) newsize <<= 1;
        std::vector<int64_t> nt(newsize, EMPTY);
        for (int64_t k : tab)
            if (k != EMPTY) put(nt, newsize - 1, k);
        tab.swap(nt);
        mask = newsize - 1;
    }
};
}  // namespace

extern "C" {

void *u2gnn_lus_create(int64_t range_max, uint32_t seed) {
    if (range_max < 1) return nullptr;
    try {
        return new Sampler(range_max, seed);
    } catch (...) {
        return nullptr;
    }
}

void u2gnn_lus_destroy(void *h) { delete static_cast<Sampler *>(h); }

int u2gnn_lus_sample(void *h, size_t size, int64_t *out_ids, int32_t *num_tries) {
    auto *s = static_cast<Sampler *>(h);
    if (!s || (!out_ids && size) || !num_tries || (int64_t)size > s->n) return -1;
    try {
        s->arena.rewind();
        IdSet data(ArenaAlloc<long>(&s->arena));
        const double log_n = std::log((double)s->n);
        int32_t tries = 0;
        while (data.size() != size) {
            ++tries;
            data.emplace(s->draw(log_n));
        }
        size_t k = 0;
        for (long v : data) out_ids[k++] = (int64_t)v;
        *num_tries = tries;
        return 0;
    } catch (const std::bad_alloc &) {
        return -2;
    } catch (...) {
        return -1;
    }
}

int u2gnn_lus_sample_pyset(void *h, size_t size, int64_t *out_ids, int32_t *num_tries) {
    auto *s = static_cast<Sampler *>(h);
    const int rc = u2gnn_lus_sample(h, size, out_ids, num_tries);
    if (rc != 0) return rc;
    try {
        PySetOrder ps(s->pytab);
        for (size_t i = 0; i < size; ++i) ps.add(out_ids[i]);
        size_t k = 0;
        for (int64_t v : s->pytab)
            if (v != PySetOrder::EMPTY) out_ids[k++] = v;
        return 0;
    } catch (const std::bad_alloc &) {
        return -2;
    }
}

int u2gnn_lus_expected_count(void *h, int32_t num_tries, const int64_t *ids, size_t n, float *out) {
    auto *s = static_cast<Sampler *>(h);
    if (!s || (n && (!ids || !out))) return -1;
    for (size_t i = 0; i < n; ++i) {
        if (ids[i] < 0 || ids[i] >= s->n) return -1;
        out[i] = (float)(-std::expm1((double)num_tries * std::log1p(-(double)s->prob[(size_t)ids[i]])));
    }
    return 0;
}

float u2gnn_lus_probability(void *h, int64_t idx) {
    auto *s = static_cast<Sampler *>(h);
    if (!s || idx < 0 || idx >= s->n) return -1.0f;
    return s->prob[(size_t)idx];
}

int u2gnn_lus_sample_unique(void *h, size_t size, const int64_t *excluded, size_t n_excluded, int64_t *out_ids) {
    auto *s = static_cast<Sampler *>(h);
    if (!s || (size && !out_ids) || (n_excluded && !excluded)) return -1;
    try {
        std::unordered_set<long> labels;
        for (size_t i = 0; i < n_excluded; ++i)
            if (excluded[i] >= 0 && excluded[i] < s->n) labels.insert((long)excluded[i]);
        if ((int64_t)size > s->n - (int64_t)labels.size()) return -1;
        std::unordered_set<long> data;
        const double log_n = std::log((double)s->n);
        while (data.size() != size) {
            const long v = s->draw(log_n);
            if (labels.find(v) == labels.end()) data.emplace(v);
        }
        size_t k = 0;
        for (long v : data) out_ids[k++] = (int64_t)v;
        return 0;
    } catch (const std::bad_alloc &) {
        return -2;
    } catch (...) {
        return -1;
    }
}

int u2gnn_lus_accidental_matches(const int64_t *labels, size_t n_labels, const int64_t *samples, size_t n_samples,
                                 int64_t *out_pairs, size_t capacity, size_t *n_out) {
    if (!n_out || (n_labels && !labels) || (n_samples && !samples)) return -1;
    try {
        std::unordered_map<long, long> pos;
        for (size_t i = 0; i < n_samples; ++i) pos[(long)samples[i]] = (long)i;
        size_t k = 0;
        for (size_t i = 0; i < n_labels; ++i) {
            auto it = pos.find((long)labels[i]);
            if (it == pos.end()) continue;
            if (k < capacity && out_pairs) {
                out_pairs[2 * k] = (int64_t)i;
                out_pairs[2 * k + 1] = (int64_t)it->second;
            }
            ++k;
        }
        *n_out = k;
        return 0;
    } catch (...) {
        return -1;
    }
}

}  // extern "C"
