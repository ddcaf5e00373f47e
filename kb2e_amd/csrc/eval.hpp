// eval.hpp -- link-prediction evaluation on the device (EmbeddingEvaluation::run,
// common/evaluation.cpp:181-251), its own translation unit (eval.hip) behind
// kb2e_evaluate / kb2e_evaluate_transr_compat.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace kb2e {

struct EvalTables {
    int32_t model;  // kb2e_model
    int32_t n, ld, ne, nr;
    int32_t l1;     // L1 distance (TransH always)
    int32_t f64;    // tables are double (else float)
    const void* ent;  // [ne][ld]
    const void* rel;  // [nr][ld]
    const void* w;    // TransH [nr][ld], TransR [nr][n][ld] ([r][j][i])
    hipStream_t stream;
};

struct EvalQuery {
    const int32_t *th, *tt, *tr;  // test triples (the reference's working set, file order)
    int64_t ntest;
    const int32_t *fh, *ft, *fr;  // filter: test + train + valid
    int64_t nfilter;
};

// Stateless energies (TransE, TransH, TransR with zeroed work vectors).
// out = raw mean rank, raw hits@10, filtered mean rank, filtered hits@10.
void evaluate_fixed(const EvalTables& t, const EvalQuery& q, double out[4]);

// TransR with the reference's accumulating energy work vectors
// (transr/transr.cpp:20-25, transr/evaluation.cpp:22-32) through its cached,
// relation-major loop (common/evaluation.cpp:107-121, 181-238).  work[2n] =
// head and tail work vectors (in: the state to start from, nullptr = zeros as
// in a fresh evalTransR; out: the state after the run).  out[4] = number of
// candidates whose energy equals the true triple's (std::sort orders those
// arbitrarily; they are ranked after the truth).  progress(fraction) is
// called after each relation.
void evaluate_transr_compat(const EvalTables& t, const EvalQuery& q, double* work, double out[5],
                            void (*progress)(double, void*) = nullptr, void* ud = nullptr);

}  // namespace kb2e
