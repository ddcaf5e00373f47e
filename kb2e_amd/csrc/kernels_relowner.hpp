// kernels_relowner.hpp -- relation-owner schedule for TransH / TransR (plan).
#pragma once

#include <algorithm>
#include <numeric>
#include <vector>

#include "host_data.hpp"
#include "kernels_common.hpp"

namespace kb2e {

// Relations are dealt to persistent "owner" workgroups by LPT bin packing on
// their training-triple counts, so the hottest relations get a workgroup of
// their own.  Every owner replays its relations' updates in global sample
// order, which is what makes the per-entity ticket protocol deadlock-free.
struct RelOwnerPlan {
    int num_owners = 0;
    std::vector<int32_t> owner;  // relation -> owner
};

inline void plan_owners(RelOwnerPlan& p, const TripleStore& ts, int num_relations, int max_owners = 256) {
    p.num_owners = std::max(1, std::min(num_relations, max_owners));
    std::vector<int> order(num_relations);
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(),
                     [&](int a, int b) { return ts.rel_count[a] > ts.rel_count[b]; });
    std::vector<int64_t> load(p.num_owners, 0);
    p.owner.assign(num_relations, 0);
    for (int r : order) {
        int best = (int)(std::min_element(load.begin(), load.end()) - load.begin());
        p.owner[r] = best;
        load[best] += ts.rel_count[r] + 1;
    }
}

}  // namespace kb2e
