/*
 * kb2e_engine.h -- the drop-in C ABI of the kb2e_amd MI355X training engine.
 *
 * The reference (eriq-augustine/KB2E) runs its per-triple SGD hot path inside
 * the C++ class common::Trainer (common/trainer.h:14-78).  Its protected
 * virtual bfgs() (common/trainer.h:59, common/trainer.cpp:69-107) loops over
 * epochs and batches, draws a corrupted triple per sample, scores both triples
 * with the model's tripleEnergy() and applies gradientUpdate() to the *_next_
 * tables (transe/trainer.cpp:25-56, transh/trainer.cpp:11-75,
 * transr/trainer.cpp:35-188).  This ABI replaces exactly that loop: a host
 * trainer overrides bfgs() and calls the functions below (INTEGRATION.md shows
 * the binding).  Everything else (argument parsing, file loading, writing the
 * embedding text files, evaluation binaries) stays on the host.
 *
 * Conventions: plain C types, caller-owned buffers borrowed only for the call,
 * row-major contiguous tables, status codes instead of exceptions.  One host
 * thread per context; contexts are independent (one per GPU / rank).
 */
#ifndef KB2E_ENGINE_H_
#define KB2E_ENGINE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    KB2E_OK = 0,
    KB2E_EINVAL = 1,      /* bad argument / shape (reference: printf + exit(1)) */
    KB2E_EDEVICE = 2,     /* HIP runtime or kernel failure */
    KB2E_ESTATE = 3,      /* call order violated (e.g. train before upload) */
    KB2E_ENOMEM = 4,
    KB2E_EUNSUPPORTED = 5,
    KB2E_ESAMPLER = 6     /* a negative could not be drawn (every entity is a
                             known triple: the reference loops forever here,
                             common/trainer.cpp:89-96) */
} kb2e_status;

typedef enum { KB2E_TRANSE = 0, KB2E_TRANSH = 1, KB2E_TRANSR = 2 } kb2e_model;

/* Where the sample stream (train index i, corrupting entity j, side) comes from. */
typedef enum {
    KB2E_SAMPLER_GLIBC = 0,  /* the reference's own stream: glibc TYPE_3 rand()
                                seeded by `seed`, consumed exactly as
                                common/trainer.cpp:79-98 (default) */
    KB2E_SAMPLER_REPLAY = 1  /* caller supplies the stream (kb2e_set_sample_stream) */
} kb2e_sampler;

/* How a batch's updates are applied to the *_next_ tables.  Both schedules
 * score every sample and compute every update direction from the
 * start-of-batch tables, as the reference does (common/trainer.cpp:130-149). */
typedef enum {
    KB2E_SCHEDULE_ORDERED = 0,  /* the reference's sequence: sample by sample, a
                                   norm after every update (transe/trainer.cpp:38-45,
                                   transh/trainer.cpp:48-58, transr/trainer.cpp:
                                   166-187); results equal the reference's (default) */
    KB2E_SCHEDULE_PARALLEL = 1  /* each touched row / relation gets its summed
                                   delta, then the model's norms and constraints
                                   once per batch; equal to ORDERED for rows with
                                   one update per batch, O(lr^2) apart otherwise.
                                   Parity is statistical (link-prediction quality,
                                   DESIGN.md) */
} kb2e_schedule;

typedef struct {
    int32_t model;          /* kb2e_model */
    int32_t dim;            /* --size (common/args.cpp:71-74) */
    int32_t num_entities;
    int32_t num_relations;
    double learning_rate;   /* --rate */
    double margin;          /* --margin */
    int32_t method;         /* 0 unif, 1 bern (common/constants.h:7-8) */
    int32_t distance;       /* 0 L1, 1 L2 (common/constants.h:16-17); TransH is always L1 */
    int32_t num_batches;    /* --batches */
    uint32_t seed;          /* --seed: srand() in main (transe/bin/trainTransE.cpp:13) */
    int32_t precision;      /* 64 = FP64 tables and arithmetic like the reference; 32 = FP32 */
    int32_t sampler;        /* kb2e_sampler */
    int32_t transr_compat;  /* 1: reproduce the accumulating TransR energy of
                               transr/transr.cpp:20-25; 0: zeroed work vectors */
    int32_t device;         /* HIP device ordinal */
    int32_t schedule;       /* kb2e_schedule */
    int32_t sub_batches;    /* PARALLEL TransR: each batch's summed updates, norms and
                               transRNorm pairs applied in this many ordered sub-batches
                               of ceil(B / k) samples (the energies, hinge decisions and
                               update directions stay on the start-of-batch tables,
                               common/trainer.cpp:132-133); nearer the reference's
                               norm after every update (transr/trainer.cpp:174-187).
                               1 = one per batch; 0 (kb2e_default_config) = by width:
                               the smallest count whose loss stays inside the
                               reference's seed envelope where measured (2 for
                               dim <= 64, 3 above).  Ignored by the other
                               models and the ORDERED schedule. */
} kb2e_config;

typedef struct kb2e_ctx kb2e_ctx;

/* Fill `cfg` with the reference defaults (common/constants.h:28-40). */
void kb2e_default_config(kb2e_config* cfg);

kb2e_status kb2e_create(const kb2e_config* cfg, kb2e_ctx** out);
/* The context's configuration with the defaults resolved (sub_batches 0 -> the
 * count the context runs). */
kb2e_status kb2e_get_config(const kb2e_ctx* ctx, kb2e_config* out);
void kb2e_destroy(kb2e_ctx* ctx);
const char* kb2e_last_error(const kb2e_ctx* ctx);

/* Trainer::add for every training triple, in train-file order, plus the
 * per-relation head/tail co-occurrence means of Trainer::loadFiles
 * (common/trainer.cpp:26-32, 151-201).  Builds the negative-sample filter and
 * the Bernoulli table on the device.  Contexts take dim <= 512 (ORDERED
 * TransR above dim 137 keeps the relation owner's matrix in L2 instead of LDS);
 * PARALLEL TransR trains dim <= 128, checked at kb2e_create
 * (KB2E_EUNSUPPORTED above). */
kb2e_status kb2e_upload_triples(kb2e_ctx* ctx, const int32_t* heads, const int32_t* tails,
                                const int32_t* relations, int64_t count);

/* Trainer::prepTrain (common/trainer.cpp:34-58; transh/trainer.cpp:77-88;
 * transr/trainer.cpp:70-86 up to the seed files): draws the initial tables from
 * the context's glibc stream exactly as the reference does, uploads them, and
 * (if the pointers are non-NULL) returns them.  Weights: TransH R x n, TransR
 * R x n x n ([r][j][i]). */
kb2e_status kb2e_init_params(kb2e_ctx* ctx, double* entity, double* relation, double* weights);

/* TransR's seed step (transr/trainer.cpp:88-113): entity rows from the
 * seed TransE run are scaled to unit length (common::norm(v, false)),
 * relation rows are taken verbatim; the relation matrices keep the identity
 * that kb2e_init_params set.  Call after kb2e_init_params. */
kb2e_status kb2e_transr_seed(kb2e_ctx* ctx, const double* entity, const double* relation);

/* Trainer::prepTrain's draws made on the device: the same
 * randn values (common/utils.cpp:26-38), row norms and TransH / TransR weight
 * init as kb2e_init_params, taken from the same glibc stream and leaving it at
 * the same position -- the epochs that follow are unchanged.  Every rejection
 * attempt is evaluated in parallel (the stream is made on the device from the
 * generator's 31-word window) and the accepted ones are compacted in order.
 * *near_ties (may be NULL) = accept/reject decisions within a few ulps of the
 * density, where the device exp and glibc's could round differently. */
kb2e_status kb2e_init_params_device(kb2e_ctx* ctx, double* entity, double* relation, double* weights,
                                    int64_t* near_ties);

/* Text tables.  table: 0 entities (|E| rows), 1 relations
 * (|R| rows), 2 weights (TransH |R| rows, TransR |R|*n rows).
 * kb2e_write_table writes the device table as Trainer::write does
 * (common/trainer.cpp:109-127, transh/trainer.cpp:94-105,
 * transr/trainer.cpp:128-142): "%.6lf\t" per value, "\n" per row, formatted
 * on the device byte for byte as glibc printf; kb2e_format_table returns the
 * same bytes in `buf` (*len = the length needed; KB2E_EINVAL if cap is short).
 * kb2e_read_table loads a table from "%lf" text as the TransR seed step reads
 * its files (transr/trainer.cpp:88-113): whitespace-separated tokens, the first
 * rows*n used, converted on the device (correctly rounded, as strtod), then
 * optionally normalised per row.  KB2E_EINVAL with the reference's message when
 * the file holds fewer numbers. */
enum { KB2E_READ_VERBATIM = 0, KB2E_READ_UNIT = 1 /* common::norm(row, false) */,
       KB2E_READ_SHRINK = 2 /* common::norm(row): only rows longer than 1 */ };
kb2e_status kb2e_write_table(kb2e_ctx* ctx, int32_t table, const char* path);
kb2e_status kb2e_format_table(kb2e_ctx* ctx, int32_t table, char* buf, int64_t cap, int64_t* len);
kb2e_status kb2e_read_table(kb2e_ctx* ctx, int32_t table, const char* path, int32_t mode);

/* Upload tables (row-major FP64 as in the reference's vectors).  `weights` may
 * be NULL for TransE.  Used for TransR seeding (transr/trainer.cpp:88-113; the
 * caller applies the entity unit norm as the reference does) and for restarts. */
kb2e_status kb2e_upload_params(kb2e_ctx* ctx, const double* entity, const double* relation,
                               const double* weights);
kb2e_status kb2e_download_params(kb2e_ctx* ctx, double* entity, double* relation, double* weights);

/* TransR energy work vectors (transr/trainer.h:28-29), for compat-mode state. */
kb2e_status kb2e_get_transr_work(kb2e_ctx* ctx, double* head_work, double* tail_work);
kb2e_status kb2e_set_transr_work(kb2e_ctx* ctx, const double* head_work, const double* tail_work);

/* KB2E_SAMPLER_REPLAY: the next `count` samples (i = train index, j = entity,
 * side = 1 corrupt tail / 0 corrupt head).  Consumed batch by batch. */
kb2e_status kb2e_set_sample_stream(kb2e_ctx* ctx, const int32_t* i, const int32_t* j,
                                   const uint8_t* side, int64_t count);

/* The sample stream of the epoch in progress (after its first batch was
 * queued): up to `count` samples in order.  Returns KB2E_ESTATE between epochs. */
kb2e_status kb2e_get_sample_stream(kb2e_ctx* ctx, int32_t* i, int32_t* j, uint8_t* side, int64_t count);

/* One epoch of Trainer::bfgs (common/trainer.cpp:72-106): numBatches batches of
 * floor(|train| / numBatches) samples.  *loss = the epoch loss the reference
 * prints at :105; *active = hinge-active samples.  Either pointer may be NULL. */
kb2e_status kb2e_train_epoch(kb2e_ctx* ctx, double* loss, int64_t* active);

/* `nbatches` batches continuing the current epoch position (wrapping into the
 * next epoch).  Asynchronous: returns once queued; results land at the next
 * kb2e_synchronize / kb2e_epoch_stats. */
kb2e_status kb2e_train_batches(kb2e_ctx* ctx, int32_t nbatches);
kb2e_status kb2e_synchronize(kb2e_ctx* ctx);
/* Loss and active count accumulated since the last call (resets them). */
kb2e_status kb2e_take_stats(kb2e_ctx* ctx, double* loss, int64_t* active);

/* Link prediction on the current device tables (EmbeddingEvaluation::run,
 * common/evaluation.cpp:181-251): for each test triple, corrupt the head and
 * the tail with every entity, rank the true triple by energy; filtered ranks
 * skip corruptions that are in the filter set (the reference passes test +
 * train + valid, common/evaluation.cpp:41-62).  out[0..3] = raw mean rank,
 * raw hits@10, filtered mean rank, filtered hits@10 (hits as fractions, as
 * printed at :249-250).  Energies are bit-identical FP64 restatements of the
 * reference's; ties with the true triple are not counted above it.  TransR
 * uses the zeroed (fixed) work vectors here; kb2e_evaluate_transr_compat is
 * the reference evalTransR's stateful energy.  Every dim a context takes
 * (kb2e_create: <= 512); the ranking itself has no limit (the query rows of a
 * rank tile are staged in LDS up to dim 600, read from L2 above). */
kb2e_status kb2e_evaluate(kb2e_ctx* ctx, const int32_t* heads, const int32_t* tails, const int32_t* relations,
                          int64_t ntest, const int32_t* filter_heads, const int32_t* filter_tails,
                          const int32_t* filter_relations, int64_t nfilter, double* out);

/* TransR as the reference's evalTransR computes it: the energy work vectors
 * are never zeroed (transr/transr.cpp:20-25, transr/evaluation.cpp:22-32), so
 * every energy depends on all energies computed before it in the evaluator's
 * cached relation-major loop (common/evaluation.cpp:107-121, 181-238; the
 * per-relation energy cache is used when |E| <= 40000, common/evaluation.h:11).
 * That sequence is replayed exactly in FP64 on the device.  `work` = 2 x dim
 * doubles (head then tail work vector): in, the state to start from (NULL =
 * zeros, as a fresh evalTransR process); out, the state after the run.
 * out[0..3] as kb2e_evaluate; out[4] = candidates whose energy equals the true
 * triple's (std::sort orders those arbitrarily, :138; they are ranked after
 * the truth here).  `progress` (may be NULL) is called after each relation
 * with the fraction of test triples done (the reference prints it, :240).
 * Every dim a context takes (W in LDS up to 140, read from L2 above). */
kb2e_status kb2e_evaluate_transr_compat(kb2e_ctx* ctx, const int32_t* heads, const int32_t* tails,
                                        const int32_t* relations, int64_t ntest, const int32_t* filter_heads,
                                        const int32_t* filter_tails, const int32_t* filter_relations,
                                        int64_t nfilter, double* work, double* out,
                                        void (*progress)(double fraction, void* user), void* user);

/* Raw glibc stream access (the context's RNG, as std::rand() in the reference). */
int32_t kb2e_rng_next(kb2e_ctx* ctx);

/* Timing of the engine's device kernels on the engine's own HIP stream (HIP
 * events around each launch; off by default).  `name` is a kernel family
 * ("score", "fold", "apply", "relowner", "index", "sample", ...).  Returns total
 * milliseconds and launch count since kb2e_profile_enable.  on = 0: off;
 * on = P >= 1: the batch kernels of every P-th batch are timed (event records
 * cost device time of their own; sampling keeps the rest of the run unperturbed),
 * per-epoch kernels always. */
kb2e_status kb2e_profile_enable(kb2e_ctx* ctx, int32_t on);
kb2e_status kb2e_profile_query(kb2e_ctx* ctx, const char* name, double* total_ms, int64_t* launches);

/* Schedule counters kept on the device (no reference counterpart: they say which
 * branch of a schedule choice ran, for tests and tools).  Synchronises the
 * context's stream.  Names: "transh_orth_rel_batches" -- PARALLEL TransH batches
 * whose normOrth relation pass ran (the gate on the previous batch's normOrth
 * work, kernels_transh_parallel.hpp); the other batches took the one-wave pass
 * alone.  KB2E_EINVAL for an unknown name. */
kb2e_status kb2e_counter(kb2e_ctx* ctx, const char* name, int64_t* value);

/* Device memory the context holds, in bytes: every device buffer it has allocated
 * and not freed (tables, epoch streams and index, exports, merge state). */
int64_t kb2e_device_bytes(const kb2e_ctx* ctx);

/* Multi-GPU epoch merge (the reference is single-process, so
 * this replaces no reference call: it is the exchange step that lets N
 * contexts, each training a head-hash shard of the triples with the
 * single-GPU schedule, act as one trainer).  At an epoch boundary every rank
 * holds T_r; the merge sets, on every rank,
 *     T <- renorm(T0 + sum_r (T_r - T0))
 * where T0 is the tables after the previous merge: the entity deltas are
 * reduce-scattered to the owner of each block of rows over RCCL, the owner
 * adds them and re-applies the model's norm constraint to the rows any rank
 * changed (as kb2e_renormalize), and an all-gather returns the merged table;
 * relation and weight deltas are all-reduced and every rank renormalises the
 * changed rows.  All work runs on the contexts' own streams; the calls return
 * when the merged tables are in place.  Two ways to build the communicator:
 *  - one process per GPU (torchrun): rank 0 makes an id with
 *    kb2e_comm_unique_id, the caller hands it to every rank (any side channel),
 *    and each rank calls kb2e_comm_init_rank (collective) and then
 *    kb2e_merge_epoch at every epoch boundary (collective);
 *  - one process driving N devices (one host thread, SURVEY.md 8(b)
 *    "Threading"): kb2e_comm_init_group over the N contexts, then
 *    kb2e_merge_epoch_group.  Contexts that all share one device (or
 *    KB2E_MERGE_LOCAL=1, which also needs one device) merge with plain device
 *    kernels instead of RCCL, which refuses two ranks on one GPU; a group that
 *    mixes shared and distinct devices is KB2E_EUNSUPPORTED.
 * Initialisation broadcasts rank 0's tables to every rank, so the ranks may
 * be created with different seeds (distinct sample streams).  The contexts must
 * agree on model, dim, table sizes and precision (kb2e_comm_init_rank checks
 * the other ranks' over the new communicator: KB2E_EINVAL on a difference);
 * their tables must be loaded (kb2e_init_params / kb2e_upload_params /
 * kb2e_transr_seed) first.  A failed init leaves the context without a
 * communicator, so it can be retried.  The N > 1 RCCL paths (several
 * processes, or ncclCommInitAll over several devices) are built for the
 * 8-GPU driver run and are not exercised on the one-GPU test box: the tests
 * cover one RCCL rank and the shared-device local backend. */
#define KB2E_COMM_ID_BYTES 128
kb2e_status kb2e_comm_unique_id(uint8_t* id /* KB2E_COMM_ID_BYTES */);
kb2e_status kb2e_comm_init_rank(kb2e_ctx* ctx, int32_t nranks, int32_t rank, const uint8_t* id);
kb2e_status kb2e_comm_init_group(kb2e_ctx* const* ctxs, int32_t n);
kb2e_status kb2e_merge_epoch(kb2e_ctx* ctx);
kb2e_status kb2e_merge_epoch_group(kb2e_ctx* const* ctxs, int32_t n);
/* This rank's place in the communicator and the entity rows it owns in the merge. */
kb2e_status kb2e_comm_info(kb2e_ctx* ctx, int32_t* nranks, int32_t* rank, int64_t* first_entity,
                           int64_t* entity_count);

/* Raw device pointers of the parameter tables (row-major, leading dimension
 * round_up(dim, 2), FP64 or FP32 by precision) and their element counts, for a
 * caller-side communicator (kb2e_amd/distributed.py: torch.distributed gloo in
 * the CPU tests). */
kb2e_status kb2e_device_tables(kb2e_ctx* ctx, void** entity, void** relation, void** weights,
                               int64_t* n_entity, int64_t* n_relation, int64_t* n_weights);
/* Re-apply the per-row norm constraints of the model, to the rows flagged
 * non-zero in the host masks (NULL = every row): TransE rows and TransH
 * entity/relation rows are shrunk to length <= 1 (common/utils.cpp:70-77),
 * TransH normals and TransR entity/relation/matrix rows scaled to unit length
 * (transh/trainer.cpp:52, transr/trainer.cpp:174-180).  Weight masks are per
 * relation. */
kb2e_status kb2e_renormalize(kb2e_ctx* ctx, const uint8_t* entity_rows, const uint8_t* relation_rows,
                             const uint8_t* weight_rows);
/* The same constraint on `count` units of one table from `first` (table 0:
 * entities, 1: relations, 2: weights, in relations), with the row mask in
 * DEVICE memory (device_mask[k] for unit first + k; NULL = every row).
 * Returns when the rows are renormalised. */
kb2e_status kb2e_renormalize_rows(kb2e_ctx* ctx, int32_t table, int64_t first, int64_t count,
                                  const uint8_t* device_mask);

#ifdef __cplusplus
}
#endif

#endif /* KB2E_ENGINE_H_ */
