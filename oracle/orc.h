/*
 * oracle/orc.h -- CPU restatement of eriq-augustine/KB2E (TEST INFRASTRUCTURE ONLY).
 *
 * This is the parity oracle for the kb2e_amd GPU engine.  It is a plain-C
 * restatement of the reference's single-threaded FP64 training and evaluation
 * loops, function by function, with the reference file:line each one follows.
 * It is pinned against golden vectors produced by the reference itself
 * (oracle/_ref/ref_harness, built from /root/reference by oracle/Makefile;
 * fixtures in tests/golden/).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library, and only as the checker / CPU baseline -- never as the product
 * path.  The product (kb2e_amd/csrc, libkb2e.so) does not link or call it.
 *
 * RNG: the reference draws from the global glibc rand() seeded by srand(seed)
 * in main() (transe/bin/trainTransE.cpp:13).  The oracle draws the same TYPE_3
 * stream through glibc's random_r on a private state, so it is bit-identical
 * to the reference on the same glibc and unaffected by other rand() callers.
 */
#ifndef KB2E_ORACLE_ORC_H_
#define KB2E_ORACLE_ORC_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORC_TRANSE = 0, ORC_TRANSH = 1, ORC_TRANSR = 2 };

typedef struct orc_model orc_model;

/* ---- L0 numerics / RNG (common/utils.cpp) ---- */
void orc_srand(unsigned seed);
int orc_rand(void);
double orc_rand_range(double min, double max);                 /* utils.cpp:18-20 */
double orc_normal(double x, double miu, double sigma);          /* utils.cpp:22-24 */
double orc_randn(double miu, double sigma, double min, double max); /* utils.cpp:26-38 */
int orc_randmax(int x);                                          /* utils.cpp:113-120 */
double orc_vec_len(const double* a, int n);                      /* utils.cpp:44-51 */
void orc_norm(double* a, int n, int ignore_short);               /* utils.cpp:70-77 */
void orc_norm_orth(double* a, double* b, int n, double rate);    /* utils.cpp:79-111 */
long long orc_norm_orth_iterations(void); /* instrumentation: loop iterations that modified a,b */
long long orc_site_iterations(int site);

/* ---- model lifecycle (common/trainer.{h,cpp}) ---- */
orc_model* orc_create(int model, int dim, int num_entities, int num_relations,
                      double learning_rate, double margin, int method, int distance,
                      int num_batches, int transr_compat);
void orc_destroy(orc_model* m);
/* Trainer::add for every triple + the co-occurrence statistics of loadFiles
 * (common/trainer.cpp:26-32, 151-201).  Triples in train-file order. */
int orc_set_triples(orc_model* m, const int* heads, const int* tails, const int* rels, int count);
/* Trainer::prepTrain (+ TransH/TransR overrides): consumes the global RNG. */
void orc_prep_train(orc_model* m);
/* TransR seed overwrite (transr/trainer.cpp:88-113): entities are unit-normed,
 * relations are copied verbatim.  `ent` is E x n, `rel` is R x n. */
void orc_transr_seed(orc_model* m, const double* ent, const double* rel);

/* Tables: entity E x n, relation R x n, weights (TransH: R x n, TransR: R x n x n
 * with [r][j][i] = weights_[r][j][i]).  get copies out, set copies in. */
void orc_get_tables(const orc_model* m, double* ent, double* rel, double* w);
void orc_set_tables(orc_model* m, const double* ent, const double* rel, const double* w);
void orc_get_transr_work(const orc_model* m, double* hwork, double* twork);
void orc_set_transr_work(orc_model* m, const double* hwork, const double* twork);

/* One epoch of Trainer::bfgs (common/trainer.cpp:69-107).  Returns the epoch
 * loss; *active receives the number of hinge-active samples. */
double orc_train_epoch(orc_model* m, long long* active);
/* Only `nbatches` batches of an epoch (for bounded CPU-baseline samples). */
double orc_train_batches(orc_model* m, int nbatches, long long* active);
/* Replay: train batches from a supplied sample stream instead of rand().
 * Samples are (i = train index, j = corrupting entity, side = 1 tail / 0 head).
 * count must be a multiple of the batch size. */
double orc_train_replay(orc_model* m, const int* si, const int* sj, const uint8_t* side,
                        long long count, long long* active);
/* The exact sample stream of the next `count` samples (consumes the RNG like
 * the sampling half of bfgs, common/trainer.cpp:79-98), without training. */
void orc_sample_stream(orc_model* m, long long count, int* si, int* sj, uint8_t* side);
int orc_batch_size(const orc_model* m);
int orc_in_train(const orc_model* m, int h, int r, int t);

/* ---- per-model kernels on the snapshot tables (KATs) ---- */
double orc_triple_energy(orc_model* m, int h, int t, int r);
/* gradientUpdate on the snapshot, writing the *_next_ tables; call
 * orc_begin_batch first (prebatch) and orc_end_batch after (postbatch). */
void orc_begin_batch(orc_model* m);
void orc_gradient_update(orc_model* m, int h, int t, int r, int corrupted);
void orc_end_batch(orc_model* m);
/* transr::Trainer::transRNorm on caller buffers (a: n, b: n x n row-major b[j][i]). */
void orc_transr_norm(double* a, double* b, int n, double rate);
long long orc_transr_norm_iterations(void);

/* ---- evaluation (common/evaluation.cpp) ---- */
/* Link prediction over `test` with filter = test + train + valid.  Mirrors
 * EmbeddingEvaluation::run (common/evaluation.cpp:181-251), including the
 * per-relation energy cache; ranks count strictly-smaller energies (ties are
 * broken in favour of the true triple; std::sort leaves tie order unspecified).
 * out[0..3] = raw mean rank, raw hits@10, filtered mean rank, filtered hits@10
 * (hits as fractions, as printed at common/evaluation.cpp:249-250);
 * out[4] = number of (query, entity) pairs whose energy ties the true triple's. */
void orc_evaluate(orc_model* m,
                  const int* th, const int* tt, const int* tr, int ntest,
                  const int* fh, const int* ft, const int* fr, int nfilter,
                  double* out);

#ifdef __cplusplus
}
#endif

#endif /* KB2E_ORACLE_ORC_H_ */
