// FilterSet's Bloom prefilter (kb2e_amd/csrc/host_data.hpp), checked on the host
// with the device sampler's probe rule (kernels_sampler.hpp filter_has): every
// training key passes (no false negatives, so the sample stream cannot change)
// and few absent keys do.  Prints "<false positives> <probes>".
#include <cstdio>
#include <random>

#include "host_data.hpp"

static bool bloom_pass(const kb2e::FilterSet& f, uint64_t k) {
    const uint64_t b = kb2e::mix64(k ^ kb2e::FilterSet::kBloomSalt);
    const uint64_t bits = (1ull << ((b >> 52) & 63)) | (1ull << (b >> 58));
    return (f.bloom[b & f.bloom_mask] & bits) == bits;
}

int main(int argc, char** argv) {
    const int ntrip = argc > 1 ? atoi(argv[1]) : 483142;
    const int ne = 14951, nr = 1345;
    std::mt19937_64 g(1);
    std::vector<int32_t> H(ntrip), T(ntrip), R(ntrip);
    for (int k = 0; k < ntrip; ++k) {
        H[k] = (int32_t)(g() % ne);
        T[k] = (int32_t)(g() % ne);
        R[k] = (int32_t)(g() % nr);
    }
    kb2e::FilterSet f;
    f.build(H, T, R, ne, nr);
    for (int k = 0; k < ntrip; ++k)
        if (!bloom_pass(f, f.key(H[k], R[k], T[k]))) {
            printf("false negative at %d\n", k);
            return 1;
        }
    long fp = 0, probes = 0;
    for (int k = 0; k < 1000000; ++k) {
        const int h = (int)(g() % ne), t = (int)(g() % ne), r = (int)(g() % nr);
        if (f.has(h, r, t)) continue;
        ++probes;
        fp += bloom_pass(f, f.key(h, r, t));
    }
    printf("%ld %ld\n", fp, probes);
    return 0;
}
