// host_data.hpp -- host-side triple store, negative filter and the
// reference-exact sample stream (common/trainer.cpp:26-32, 79-98, 151-201).
#pragma once

#include <algorithm>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "glibc_rand.hpp"

namespace kb2e {

inline uint64_t mix64(uint64_t x) {
    x ^= x >> 31;
    x *= 0x7fb5d329728ea185ull;
    x ^= x >> 27;
    x *= 0x81dadef4bc2dd44dull;
    x ^= x >> 33;
    return x;
}

// Open-addressing set of (head, relation, tail) keys: the reference's
// triples_ map used as "is this corrupted triple a known training triple"
// (common/trainer.h:49, queried at common/trainer.cpp:89 and :94).  The same
// table (power-of-two slots, linear probing, empty = ~0) is uploaded to HBM
// for the device sampler.
struct FilterSet {
    std::vector<uint64_t> slots;
    uint64_t mask = 0;
    uint64_t ne = 1, nr = 1;
    // Blocked Bloom prefilter for the device sampler (>= 12 bits a key, two bits
    // in one 64-bit word): a corrupted triple almost never is a training triple,
    // so sample_len answers most probes from this L2-sized array instead of a
    // random line of `slots`.  No false negatives: results are unchanged.
    std::vector<uint64_t> bloom;
    uint64_t bloom_mask = 0;

    static constexpr uint64_t kEmpty = ~0ull;
    static constexpr uint64_t kBloomSalt = 0x9e3779b97f4a7c15ull;

    uint64_t key(int64_t h, int64_t r, int64_t t) const {
        return ((uint64_t)h * nr + (uint64_t)r) * ne + (uint64_t)t;
    }

    void build(const std::vector<int32_t>& H, const std::vector<int32_t>& T,
               const std::vector<int32_t>& R, int64_t num_entities, int64_t num_relations) {
        ne = (uint64_t)num_entities;
        nr = (uint64_t)num_relations;
        uint64_t cap = 16;
        while (cap < 2 * (uint64_t)H.size() + 16) cap <<= 1;
        slots.assign(cap, kEmpty);
        mask = cap - 1;
        for (size_t k = 0; k < H.size(); ++k) insert(key(H[k], R[k], T[k]));
        uint64_t nw = 64;
        while (nw * 64 < 12 * (uint64_t)H.size()) nw <<= 1;
        bloom.assign(nw, 0);
        bloom_mask = nw - 1;
        for (size_t k = 0; k < H.size(); ++k) {
            const uint64_t b = mix64(key(H[k], R[k], T[k]) ^ kBloomSalt);
            bloom[b & bloom_mask] |= (1ull << ((b >> 52) & 63)) | (1ull << (b >> 58));
        }
    }

    void insert(uint64_t k) {
        uint64_t p = mix64(k) & mask;
        while (slots[p] != kEmpty) {
            if (slots[p] == k) return;
            p = (p + 1) & mask;
        }
        slots[p] = k;
    }

    bool has(int64_t h, int64_t r, int64_t t) const {
        uint64_t k = key(h, r, t);
        uint64_t p = mix64(k) & mask;
        while (true) {
            uint64_t s = slots[p];
            if (s == k) return true;
            if (s == kEmpty) return false;
            p = (p + 1) & mask;
        }
    }
};

struct TripleStore {
    int32_t ne = 0, nr = 0;
    std::vector<int32_t> heads, tails, rels;
    FilterSet filter;
    std::vector<double> pr;           // 1000 * tailMean / (tailMean + headMean) per relation
    std::vector<int32_t> rel_count;   // training triples per relation
    std::vector<int32_t> max_tails;   // max #distinct tails of any (h, r) (rejection bound check)

    void build(const int32_t* h, const int32_t* t, const int32_t* r, int64_t count,
               int32_t num_entities, int32_t num_relations) {
        ne = num_entities;
        nr = num_relations;
        heads.assign(h, h + count);
        tails.assign(t, t + count);
        rels.assign(r, r + count);
        for (int64_t k = 0; k < count; ++k) {
            if (h[k] < 0 || h[k] >= ne || t[k] < 0 || t[k] >= ne || r[k] < 0 || r[k] >= nr)
                throw std::invalid_argument("triple " + std::to_string(k) + " has an id out of range");
        }
        filter.build(heads, tails, rels, ne, nr);
        // Trainer::loadFiles co-occurrence means (common/trainer.cpp:163-194):
        // per relation, mean over distinct heads (tails) of their triple count.
        std::vector<double> hmean(nr, 0.0), tmean(nr, 0.0);
        rel_count.assign(nr, 0);
        for (int side = 0; side < 2; ++side) {
            std::vector<uint64_t> pairs((size_t)count);
            for (int64_t k = 0; k < count; ++k)
                pairs[k] = ((uint64_t)(uint32_t)r[k] << 32) | (uint32_t)(side == 0 ? h[k] : t[k]);
            std::sort(pairs.begin(), pairs.end());
            std::vector<double>& out = side == 0 ? hmean : tmean;
            size_t k = 0;
            while (k < pairs.size()) {
                uint32_t rel = (uint32_t)(pairs[k] >> 32);
                double total = 0;
                int64_t distinct = 0;
                while (k < pairs.size() && (uint32_t)(pairs[k] >> 32) == rel) {
                    size_t e = k;
                    while (e < pairs.size() && pairs[e] == pairs[k]) ++e;
                    ++distinct;
                    total += (double)(e - k);
                    k = e;
                }
                out[rel] = total / (double)distinct;
                if (side == 0) rel_count[rel] = (int32_t)total;
            }
        }
        pr.assign(nr, 0.0);
        for (int i = 0; i < nr; ++i) pr[i] = 1000 * tmean[i] / (tmean[i] + hmean[i]);
    }

    int64_t size() const { return (int64_t)heads.size(); }
};

// The sampling half of Trainer::bfgs (common/trainer.cpp:79-98) on the host:
// i = randMax(|train|), j = randMax(|E|), then rand() % 1000 against pr (500
// for unif), then rejection of known triples.  Returns false if a rejection
// loop cannot terminate (every entity completes the triple).
struct HostSampler {
    static constexpr int64_t kMaxRejections = 50'000'000;

    static bool draw(GlibcRand& g, const TripleStore& ts, int method, int32_t& si, int32_t& sj,
                     uint8_t& side) {
        int32_t i = rand_max(g, (int32_t)ts.size());
        int32_t j = rand_max(g, ts.ne);
        int32_t r = ts.rels[i];
        double pr = ts.pr[r];
        if (method == 0) pr = 500;
        int64_t spins = 0;
        if (g.next() % 1000 < pr) {
            while (ts.filter.has(ts.heads[i], r, j)) {
                j = rand_max(g, ts.ne);
                if (++spins > kMaxRejections) return false;
            }
            side = 1;
        } else {
            while (ts.filter.has(j, r, ts.tails[i])) {
                j = rand_max(g, ts.ne);
                if (++spins > kMaxRejections) return false;
            }
            side = 0;
        }
        si = i;
        sj = j;
        return true;
    }
};

}  // namespace kb2e
