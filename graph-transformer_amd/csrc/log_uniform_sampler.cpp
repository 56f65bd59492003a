// Host-side log-uniform sampler for the sampled-softmax loss (C ABI: include/u2gnn_lus.h).
// A new implementation of the reference's sampler contract (see the header for citations);
// it keeps the reference's engine and set semantics so the drawn ids are identical.
#include "u2gnn_lus.h"

#include <cmath>
#include <new>
#include <random>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace {
struct Sampler {
    int64_t n;
    std::minstd_rand0 engine;                    // == std::default_random_engine (libstdc++)
    std::uniform_real_distribution<double> uni;  // [0, 1)
    std::vector<float> prob;
    Sampler(int64_t n_, uint32_t seed) : n(n_), engine(seed), uni(0.0, 1.0), prob((size_t)n_) {
        const double lr = std::log((double)(n_ + 1));
        for (int64_t i = 0; i < n_; ++i) prob[(size_t)i] = (float)((std::log((double)(i + 2)) - std::log((double)(i + 1))) / lr);
    }
    long draw(double log_n) { return std::lround(std::exp(uni(engine) * log_n)) - 1; }
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
        std::unordered_set<long> data;
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
