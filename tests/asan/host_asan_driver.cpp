// AddressSanitizer / UBSan driver for the host natives of libu2gnn_lus.so:
// csrc/batch_assembly.cpp and csrc/log_uniform_sampler.cpp are compiled into this program with
// -fsanitize=address,undefined (tests/test_asan_cpu.py builds and runs it), fed the cases the
// Python test writes (int64 records), and their outputs written back for comparison with the
// regular build.  Any out-of-bounds access to the caller's CSR / MT state / output arrays aborts.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "u2gnn_lus.h"

namespace {

struct In {
    FILE *f;
    int64_t get() {
        int64_t v;
        if (std::fread(&v, 8, 1, f) != 1) throw 1;
        return v;
    }
    std::vector<int64_t> vec(int64_t n) {
        std::vector<int64_t> v((size_t)n);   // exact size: ASan sees any overrun
        if (n && std::fread(v.data(), 8, (size_t)n, f) != (size_t)n) throw 1;
        return v;
    }
};

struct Out {
    FILE *f;
    void put(int64_t v) { std::fwrite(&v, 8, 1, f); }
    void vec(const int64_t *p, int64_t n) {
        put(n);
        if (n) std::fwrite(p, 8, (size_t)n, f);
    }
};

void assembly_case(In &in, Out &out) {
    std::vector<int64_t> key64 = in.vec(624);
    std::vector<uint32_t> key(624);
    for (int i = 0; i < 624; ++i) key[i] = (uint32_t)key64[i];
    int32_t pos = (int32_t)in.get();
    const int64_t n_ids = in.get();
    std::vector<int64_t> ids = in.vec(n_ids);
    const int64_t G = in.get();
    std::vector<int64_t> n_nodes = in.vec(G), node_start = in.vec(G + 1);
    const int64_t V = in.get();
    std::vector<int64_t> deg = in.vec(V), nbr_start = in.vec(V + 1);
    const int64_t E = in.get();
    std::vector<int64_t> nbr = in.vec(E);
    const int32_t k = (int32_t)in.get();
    const int64_t n_cap = in.get();
    std::vector<int64_t> offsets((size_t)n_ids + 1), input_x((size_t)(n_cap * (k + 1))), gnode((size_t)n_cap);
    const int rc = u2gnn_batch_assemble(key.data(), &pos, ids.data(), n_ids, n_nodes.data(), node_start.data(),
                                        deg.data(), nbr_start.data(), nbr.data(), k, n_cap, offsets.data(),
                                        input_x.data(), gnode.data());
    out.put(rc);
    const int64_t N = rc == 0 ? offsets[(size_t)n_ids] : 0;
    out.vec(offsets.data(), rc == 0 ? n_ids + 1 : 0);
    out.vec(input_x.data(), N * (k + 1));
    out.vec(gnode.data(), N);
    for (int i = 0; i < 624; ++i) key64[i] = key[i];
    out.vec(key64.data(), 624);
    out.put(pos);
}

void sampler_case(In &in, Out &out) {
    const int64_t N = in.get(), seed = in.get(), size = in.get(), reps = in.get();
    const int64_t n_excl = in.get();
    std::vector<int64_t> excl = in.vec(n_excl);
    void *h = u2gnn_lus_create(N, (uint32_t)seed);
    std::vector<int64_t> ids((size_t)size);
    for (int64_t r = 0; r < reps; ++r) {
        int32_t tries = 0;
        const int rc = u2gnn_lus_sample(h, (size_t)size, ids.data(), &tries);
        out.put(rc);
        out.put(tries);
        out.vec(ids.data(), rc == 0 ? size : 0);
        std::vector<float> ec((size_t)size);
        std::vector<int64_t> ecb((size_t)size);
        const int rc2 = rc == 0 ? u2gnn_lus_expected_count(h, tries, ids.data(), (size_t)size, ec.data()) : -1;
        for (int64_t i = 0; i < size; ++i) {
            uint32_t b;
            std::memcpy(&b, &ec[(size_t)i], 4);
            ecb[(size_t)i] = b;
        }
        out.put(rc2);
        out.vec(ecb.data(), rc2 == 0 ? size : 0);
    }
    const int rc3 = u2gnn_lus_sample_unique(h, (size_t)size, excl.data(), (size_t)n_excl, ids.data());
    out.put(rc3);
    out.vec(ids.data(), rc3 == 0 ? size : 0);
    std::vector<int64_t> pairs((size_t)(2 * n_excl * size + 2));
    size_t n_out = 0;
    const int rc4 = u2gnn_lus_accidental_matches(excl.data(), (size_t)n_excl, ids.data(), rc3 == 0 ? (size_t)size : 0,
                                                 pairs.data(), (size_t)(n_excl * size + 1), &n_out);
    out.put(rc4);
    out.vec(pairs.data(), rc4 == 0 ? (int64_t)(2 * n_out) : 0);
    u2gnn_lus_destroy(h);
}

}  // namespace

int main(int argc, char **argv) {
    if (argc != 3) {
        std::fprintf(stderr, "usage: host_asan_driver IN OUT\n");
        return 2;
    }
    In in{std::fopen(argv[1], "rb")};
    Out out{std::fopen(argv[2], "wb")};
    if (!in.f || !out.f) return 2;
    try {
        const int64_t n_asm = in.get(), n_lus = in.get();
        for (int64_t i = 0; i < n_asm; ++i) assembly_case(in, out);
        for (int64_t i = 0; i < n_lus; ++i) sampler_case(in, out);
    } catch (int) {
        std::fprintf(stderr, "short input\n");
        return 3;
    }
    std::fclose(out.f);
    return 0;
}
