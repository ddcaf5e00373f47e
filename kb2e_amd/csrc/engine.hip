// engine.hip -- kb2e_amd training engine: C ABI (include/kb2e_engine.h) and
// per-epoch orchestration on one MI355X.
//
// Per epoch (Trainer::bfgs, common/trainer.cpp:69-107):
//   1. sample stream: the reference's exact glibc stream (host sampler) or a
//      replayed one, uploaded once per epoch;
//   2. event index: one key per (row, sample, update) event, radix-sorted by
//      (batch, row, sample) and cut into per-row segments (kernels_index.hpp);
//   3. per batch: phase A (score: energies, hinge, update directions from the
//      start-of-batch tables) then phase B (ordered per-row folds for TransE;
//      relation-owner schedule for TransH/TransR) -- the reference's
//      prebatch/postbatch snapshot semantics without any table copies.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/kb2e_engine.h"
#include "glibc_rand.hpp"
#include "hip_util.hpp"
#include "eval.hpp"
#include "host_data.hpp"
#include "kernels_common.hpp"
#include "kernels_index.hpp"
#include "kernels_transe.hpp"
#include "kernels_transe_long.hpp"
#include "kernels_relowner.hpp"
#include "kernels_sampler.hpp"
#include "kernels_parallel.hpp"
#include "kernels_transr_parallel.hpp"
#include "kernels_transr_mfma.hpp"
#include "transr_cons.hpp"
#include "kernels_transh_parallel.hpp"
#include "textio.hpp"

using namespace kb2e;

namespace {

constexpr int kGlibcBlock = 4096;  // words per block of the device glibc generator

int bits_for(int64_t v) {  // bits to hold values 0..v
    int b = 1;
    while ((1ll << b) <= v) ++b;
    return b;
}

struct Timer {
    double ms = 0;
    int64_t launches = 0;
};

}  // namespace

struct kb2e_ctx;
struct MergeState;               // engine_merge.inc
void merge_free(MergeState* m);  // engine_merge.inc
namespace {
void setup_relowner_buffers(kb2e_ctx* c);
template <typename T>
void run_batch_relowner(kb2e_ctx* c, int64_t b);
void check_dataflow(kb2e_ctx* c);
void build_owner_index(kb2e_ctx* c);
void prepare_relowner_kernels();
void setup_transr_parallel(kb2e_ctx* c);
void build_transr_tiles(kb2e_ctx* c, bool tiles, hipStream_t st, int set);
template <typename T>
void run_batch_transr_parallel(kb2e_ctx* c, int64_t b);
template <typename T, int CH>
void run_batch_transh_parallel(kb2e_ctx* c, int64_t b);
}  // namespace

struct kb2e_ctx {
    // live DevBuf bytes charged to this context (DevBuf::tally; first, so it outlives
    // every buffer member's destructor)
    int64_t device_bytes = 0;
    kb2e_config cfg{};
    std::string err;
    GlibcRand rng{1};
    TripleStore ts;
    DevBuf rel_order;  // relation ids by training frequency, most frequent first
    bool have_triples = false, have_params = false;
    int tables_read = 0;  // kb2e_read_table: bit t = table t loaded from text
    int n = 0, ld = 0, ch = 1, nw = 2, esize = 8;
    int64_t B = 0, nb = 0, S = 0;
    // PARALLEL TransR sub-batches (kb2e_config.sub_batches): index batches a batch, their
    // size (the last one the rest) and count (nbi = nb * sub; 1, B, nb otherwise)
    int32_t sub = 1;
    int64_t Bs = 0, nbi = 0;
    DevBuf snap_ent, snap_rel, snap_w;  // the start-of-batch tables phase A reads (sub > 1)
    // sub > 1: the second set of phase A's exports (phase A of sub-batch j + 1 runs on
    // suba_stream beside phase B of sub-batch j) and the events that order them
    DevBuf sb_x, sb_d, sb_y, sb_wpart, sb_rpart, sb_pflag, sb_cons_tile, sb_cpairs, sb_vio, sb_cnrows;
    hipStream_t suba_stream = nullptr;
    hipEvent_t ev_adone[2] = {nullptr, nullptr}, ev_bdone[2] = {nullptr, nullptr};
    uint64_t wait_ticks = 0;            // relation-owner ticket waits: wall-clock bound (engine_relowner.inc)
    hipStream_t stream = nullptr;

    // tables (real_t = double or float by cfg.precision)
    DevBuf ent, rel, w;
    int64_t w_elems = 0;  // logical elements (TransH R*n, TransR R*n*n)
    // triples
    DevBuf heads, tails, rels;
    // epoch sample stream, double-buffered: set `cur` feeds the epoch being
    // trained, set cur^1 receives the next epoch's stream (device sampler).
    DevBuf si_[2], sj_[2], side_[2];
    int cur = 0;
    int32_t* pin_si = nullptr;
    int32_t* pin_sj = nullptr;
    uint8_t* pin_side = nullptr;
    // device sampler (KB2E_SAMPLER_GLIBC): raw words of the glibc stream are
    // made on the host, the rejection chain is resolved on the device.
    hipStream_t side_stream = nullptr;
    DevBuf words, levels, jfin, sidefin, filter_slots, filter_bloom, pr_dev, consumed_dev;
    DevBuf trip;  // int4 per training triple: head, tail, relation, Bernoulli threshold (sample_len),
                  // or packed in 8 bytes when the ids fit (trip_eb > 0; SamplerArgs::trip8)
    int32_t trip_eb = 0, trip_rb = 0;
    DevBuf glibc_pow;  // M^(2^k) of the kGlibcBlock-word jump (glibc_starts_pow_kernel)
    DevBuf chain_table, chain_super, chain_sc, chain_ch, chain_overflow;  // the chain by chunks
    bool sampler_doubling = false;  // a sample longer than kChainEmax words was seen: pointer doubling
    int64_t* pin_consumed = nullptr;
    uint32_t* pin_win = nullptr;            // generator window after the epoch (31 words)
    DevBuf raw_words, glibc_starts, glibc_table, win_dev;
    int64_t nraw = 0, nraw_cap = 0;
    int levels_cap = 0;  // next[] levels the sampler buffers hold (1, or log S for pointer doubling)
    double words_per_sample = 6.0;
    bool prefetch_valid = false;   // set cur^1 holds the stream for the current rng state
    uint64_t rng_version = 0, prefetch_version = 0;
    // PARALLEL schedule: the next epoch's event index is built on the side stream
    // right after its sample stream, into the shadow buffers (sh_*), and swapped in
    // at the epoch boundary (swap_index) -- no index build on the batches' stream
    int64_t prefetch_gen = 0, committed_gen = -1, index_pre_gen = -2;
    bool next_pending = false;  // launch_next after the epoch's first batch
    hipEvent_t ev_index = nullptr;
    hipEvent_t ev_sampled = nullptr, ev_epoch_done = nullptr;
    bool host_sampler = false;     // KB2E_HOST_SAMPLER=1: draw on the host (debug)
    // replay stream supplied by the caller
    std::vector<int32_t> rp_si, rp_sj;
    std::vector<uint8_t> rp_side;
    int64_t rp_pos = 0;
    // event index
    KeyLayout kl{};
    int slots = 6;
    DevBuf keys, keys_sorted, sort_tmp, flags, idx, seg_start, nseg, nvalid, batch_seg;
    size_t sort_tmp_bytes = 0, scan_tmp_bytes = 0;
    // phase A outputs
    DevBuf act, loss;      // [S]
    DevBuf xbits, xreal;   // [B][2][nw], [B][2][ld]
    DevBuf aux, aux2;      // model-specific per-update exports
    // relation-owner schedule (TransH / TransR)
    RelOwnerPlan plan;
    DevBuf owner, tickets, ent_done, wsnap, transr_work, transr_work_alt, owner_seg, dataflow_err, wtouched, desc, cdesc, ocount;
    int num_cus = 256;
    uint32_t batch_stamp = 0;
    uint32_t rpar_ptab_mask = 0;
    int32_t gram_min = 48;  // KB2E_GRAM_MIN: fold segments this long use the scalar recurrence (0 = off)
    int32_t long_min = 192;  // KB2E_FOLD_LONG: segments this long take the 4-wave fold (0 = off; L1 only)
    int32_t apply_long_min = 256;  // KB2E_APPLY_LONG: PARALLEL-schedule segments this long take a 16-wave workgroup
    int32_t par_long_cap = 1, apply_grid = 256;
    DevBuf par_long_list, par_long_count;  // per epoch: long segments of every batch
    DevBuf hpar_orth;                      // PARALLEL TransH: orthogonality flags per sample
    DevBuf hpar_ids;                       // ... and a flagged sample's ids [B][8]
    DevBuf hpar_tag;                       // PARALLEL TransH: per entity, the relations its flagged pairs have
    uint32_t hpar_stamp = 0;
    DevBuf hpar_clk;                       // KB2E_HPAR_CLK: the w-apply workgroups' clocks (diagnostic)
    DevBuf hpar_count;                     // PARALLEL TransH: normOrth iterations of the last two batches, relation passes run
    uint32_t hpar_orth_min = 0;            // ... from which normOrth takes the relation pass
    int32_t hpar_orth_q = 0;               // the one-wave pass's second-sweep queue (kOrthQ)
    // PARALLEL schedule: per-event records in sorted order (kernels_transe.hpp EventRecs)
    DevBuf ev_iota, ev_slot_sorted, ev_inv, seg_row, ev_meta, ev_words;
    // PARALLEL TransR (kernels_transr_parallel.hpp)
    int32_t rpar_St = 8, rpar_max_tiles = 1, rpar_tile_threads = 256, rpar_tgroup = 1;
    bool rpar_no_constraint = false;
    bool rpar_mfma = false;  // matrix-core tile kernels (kernels_transr_mfma.hpp)
    bool rpar_cons_wave = false;  // transRNorm rounds in one wave's registers (kernels_transr_cons.hpp)
    size_t rpar_cons_lds = 0;
    bool rpar_cons_seq = false;   // transRNorm per relation, a chain of chunks (kernels_transr_seq.hpp)
    size_t rpar_seq_lds = 0;
    DevBuf rpar_vio;              // the n <= 64 chain kernels' violator slots (in-kernel pair records)
    bool rpar_cons_wide = false;  // the same chain for n <= 112 off the n <= 64 matrix-core path (kernels_transr_chainw.hpp)
    size_t rpar_wide_lds = 0;
    bool rpar_cons_gen = false;   // the same chain for FP32 and 112 < n <= 128 (kernels_transr_chaing.hpp)
    size_t rpar_gen_lds = 0;
    bool rpar_widep = false;      // 128 < n <= 512: the whole step in kernels_transr_widep.hpp
    WideGeom rpar_wg;             // (its tile / scan geometry and LDS sizes)
    DevBuf rpar_wsc;              // its transRNorm chains' W_c images, a workgroup's each
    DevBuf rpar_pflag, rpar_cons_tile, rpar_cpairs, rpar_cnrows;
    DevBuf rpar_y, rpar_wpart, rpar_rpart, rpar_tile_act, rpar_pair, rpar_relpair, rpar_relpair_stamp, rpar_scan_pre, rpar_tiles,
        rpar_ntiles, rpar_tile_first, rpar_rel_begin, rpar_scan;
    DevBuf rpar_ptab;  // transRNorm pair dedupe: two per-batch (relation, entity) tables
    DevBuf rpar_batch_t0, rpar_td_r, rpar_td_cnt, rpar_td_kk, rpar_td_ent;  // per-epoch tile descriptors
    DevBuf sh_rpar_batch_t0, sh_rpar_td_r, sh_rpar_td_cnt, sh_rpar_td_kk, sh_rpar_td_ent;
    // per batch: the relations it holds, most frequent first (the chain kernels' blocks), and
    // their count, copied to pinned host memory with the index (the chain launches' grids)
    DevBuf rpar_brel, sh_rpar_brel, rpar_bnrel, sh_rpar_bnrel;
    int64_t rpar_brel_cap = 0;
    int32_t* pin_bnrel = nullptr;
    int32_t* pin_sh_bnrel = nullptr;
    hipStream_t fold_stream = nullptr;  // the long-segment fold runs beside the per-row fold
    hipEvent_t ev_fold_a = nullptr, ev_fold_b = nullptr;
    DevBuf long_list, long_count;
    DevBuf sh_keys, sh_keys_sorted, sh_sort_tmp, sh_flags, sh_idx, sh_seg_start, sh_nseg, sh_nvalid, sh_batch_seg,
        sh_ev_slot_sorted, sh_ev_inv, sh_seg_row, sh_rpar_ntiles, sh_rpar_rel_begin, sh_rpar_tile_first,
        sh_rpar_tiles, sh_par_long_list, sh_par_long_count;
    // stats
    DevBuf stats;  // double loss, double active (reduced)
    double acc_loss = 0;
    int64_t acc_active = 0;
    int64_t reduced_upto = 0;  // samples of the current epoch already reduced
    // position
    int64_t epoch_pos = 0;  // next batch within the epoch
    bool epoch_ready = false;
    // profiling
    bool prof = false;
    int32_t prof_period = 1;   // time the batch kernels of every prof_period-th batch
    int64_t prof_counter = 0;
    bool prof_batch = true;    // the batch being queued is timed
    std::map<std::string, Timer> timers;
    struct Pending {
        std::string name;
        hipEvent_t a, b;
    };
    std::vector<Pending> pending;
    std::vector<hipEvent_t> event_pool;
    // multi-GPU epoch merge (engine_merge.inc): communicator, base tables, buffers
    MergeState* mg = nullptr;

    ~kb2e_ctx() {
        if (mg) merge_free(mg);
        if (pin_si) (void)hipHostFree(pin_si);
        if (pin_sj) (void)hipHostFree(pin_sj);
        if (pin_side) (void)hipHostFree(pin_side);
        if (pin_win) (void)hipHostFree(pin_win);
        if (pin_consumed) (void)hipHostFree(pin_consumed);
        if (pin_bnrel) (void)hipHostFree(pin_bnrel);
        if (pin_sh_bnrel) (void)hipHostFree(pin_sh_bnrel);
        flush_timers();
        if (ev_sampled) (void)hipEventDestroy(ev_sampled);
        if (ev_epoch_done) (void)hipEventDestroy(ev_epoch_done);
        if (ev_index) (void)hipEventDestroy(ev_index);
        if (side_stream) (void)hipStreamDestroy(side_stream);
        if (suba_stream) (void)hipStreamDestroy(suba_stream);
        for (hipEvent_t e : {ev_adone[0], ev_adone[1], ev_bdone[0], ev_bdone[1]})
            if (e) (void)hipEventDestroy(e);
        if (fold_stream) (void)hipStreamDestroy(fold_stream);
        if (ev_fold_a) (void)hipEventDestroy(ev_fold_a);
        if (ev_fold_b) (void)hipEventDestroy(ev_fold_b);
        for (auto e : event_pool) (void)hipEventDestroy(e);
        if (stream) (void)hipStreamDestroy(stream);
    }

    bool f64() const { return cfg.precision == 64; }
    bool parallel() const { return cfg.schedule == KB2E_SCHEDULE_PARALLEL; }
    int32_t* si() const { return si_[cur].as<int32_t>(); }
    int32_t* sj() const { return sj_[cur].as<int32_t>(); }
    uint8_t* side() const { return side_[cur].as<uint8_t>(); }

    hipEvent_t get_event() {
        if (!event_pool.empty()) {
            hipEvent_t e = event_pool.back();
            event_pool.pop_back();
            return e;
        }
        hipEvent_t e;
        HIPCHK(hipEventCreate(&e));
        return e;
    }

    // Bracket a launch with events on the engine stream (when profiling).
    template <class F>
    void timed(const char* name, F&& f) {
        timed_on(stream, name, f);
    }
    // A span of work on the engine stream (e.g. several concurrent kernels
    // joined back into it), timed from begin_span() to end_span().
    hipEvent_t begin_span() {
        if (!prof || !prof_batch) return nullptr;
        hipEvent_t a = get_event();
        HIPCHK(hipEventRecord(a, stream));
        return a;
    }
    void end_span(const char* name, hipEvent_t a) {
        if (!a) return;
        hipEvent_t b = get_event();
        HIPCHK(hipEventRecord(b, stream));
        pending.push_back({name, a, b});
    }
    // ... or on another stream that the engine stream later waits for.
    template <class F>
    void timed_on(hipStream_t st, const char* name, F&& f) {
        if (!prof || !prof_batch) {
            f();
            return;
        }
        hipEvent_t a = get_event(), b = get_event();
        HIPCHK(hipEventRecord(a, st));
        f();
        HIPCHK(hipEventRecord(b, st));
        pending.push_back({name, a, b});
        if (pending.size() > 4096) flush_timers();
    }

    // Kernel-timestamp timing (hipExtLaunchKernelGGL): the start / stop events
    // are taken at the kernel's own start and end, not around its dispatch, so
    // the averages match rocprofv3's kernel durations.  ev_begin() gives the
    // start event of a span (first kernel) and ev_end() its stop event (last
    // kernel); both null when this batch is not sampled.
    hipEvent_t span_a = nullptr;
    const char* span_name = nullptr;
    void ev_begin(const char* name, hipEvent_t& a) {
        a = nullptr;
        if (!prof || !prof_batch) return;
        a = span_a = get_event();
        span_name = name;
    }
    void ev_end(hipEvent_t& b) {
        b = nullptr;
        if (!span_a) return;
        b = get_event();
        pending.push_back({span_name, span_a, b});
        span_a = nullptr;
    }
    template <typename... KArgs, typename... Args>
    void launch(void (*kernel)(KArgs...), dim3 grid, dim3 block, size_t lds, hipEvent_t a, hipEvent_t b,
                Args... args) {
        if (a || b) hipExtLaunchKernelGGL(kernel, grid, block, lds, stream, a, b, 0, args...);
        else hipLaunchKernelGGL(kernel, grid, block, lds, stream, args...);
        HIPCHK(hipGetLastError());
    }

    void flush_timers() {
        if (pending.empty()) return;
        (void)hipStreamSynchronize(stream);
        for (auto& p : pending) {
            float ms = 0;
            if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
                timers[p.name].ms += ms;
                timers[p.name].launches += 1;
            }
            event_pool.push_back(p.a);
            event_pool.push_back(p.b);
        }
        pending.clear();
    }
};

namespace {

kb2e_status fail(kb2e_ctx* c, kb2e_status s, const std::string& msg) {
    if (c) c->err = msg;
    return s;
}

// the device buffers an entry point allocates are charged to its context
struct TallyScope {
    int64_t* prev;
    explicit TallyScope(int64_t* t) : prev(DevBuf::tally_now) { DevBuf::tally_now = t; }
    ~TallyScope() { DevBuf::tally_now = prev; }
};

template <class F>
kb2e_status guarded(kb2e_ctx* c, F&& f) {
    if (!c) return KB2E_EINVAL;
    TallyScope ts(&c->device_bytes);
    try {
        return f();
    } catch (const HipError& e) {
        return fail(c, KB2E_EDEVICE, e.what());
    } catch (const Unsupported& e) {
        return fail(c, KB2E_EUNSUPPORTED, e.what());
    } catch (const std::invalid_argument& e) {
        return fail(c, KB2E_EINVAL, e.what());
    } catch (const std::bad_alloc&) {
        return fail(c, KB2E_ENOMEM, "host out of memory");
    } catch (const std::exception& e) {
        return fail(c, KB2E_EDEVICE, e.what());
    }
}

// ------------------------------------------------------------ table transfer

template <typename T>
void upload_rows(kb2e_ctx* c, DevBuf& dst, const double* src, int64_t rows, int n, int ld) {
    std::vector<T> tmp((size_t)rows * ld, T(0));
    for (int64_t r = 0; r < rows; ++r)
        for (int i = 0; i < n; ++i) tmp[(size_t)r * ld + i] = (T)src[(size_t)r * n + i];
    HIPCHK(hipMemcpyAsync(dst.p, tmp.data(), tmp.size() * sizeof(T), hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
}

template <typename T>
void download_rows(kb2e_ctx* c, const DevBuf& src, double* dst, int64_t rows, int n, int ld) {
    std::vector<T> tmp((size_t)rows * ld);
    HIPCHK(hipMemcpyAsync(tmp.data(), src.p, tmp.size() * sizeof(T), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    for (int64_t r = 0; r < rows; ++r)
        for (int i = 0; i < n; ++i) dst[(size_t)r * n + i] = (double)tmp[(size_t)r * ld + i];
}

int64_t w_rows(const kb2e_ctx* c) {
    if (c->cfg.model == KB2E_TRANSH) return c->cfg.num_relations;
    if (c->cfg.model == KB2E_TRANSR) return (int64_t)c->cfg.num_relations * c->n;
    return 0;
}

void sync_wsnap(kb2e_ctx* c) {
    if (c->cfg.model != KB2E_TRANSR) return;
    HIPCHK(hipMemcpyAsync(c->wsnap.p, c->w.p, c->w.bytes, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
}

void upload_tables(kb2e_ctx* c, const double* e, const double* r, const double* w) {
    const int64_t ne = c->cfg.num_entities, nr = c->cfg.num_relations;
    if (c->f64()) {
        if (e) upload_rows<double>(c, c->ent, e, ne, c->n, c->ld);
        if (r) upload_rows<double>(c, c->rel, r, nr, c->n, c->ld);
        if (w && w_rows(c)) upload_rows<double>(c, c->w, w, w_rows(c), c->n, c->ld);
    } else {
        if (e) upload_rows<float>(c, c->ent, e, ne, c->n, c->ld);
        if (r) upload_rows<float>(c, c->rel, r, nr, c->n, c->ld);
        if (w && w_rows(c)) upload_rows<float>(c, c->w, w, w_rows(c), c->n, c->ld);
    }
    if (w) sync_wsnap(c);
}

// ------------------------------------------------------------------- index

// The index buffers of one epoch (build_index writes them; the batches read them).
std::vector<std::pair<DevBuf*, DevBuf*>> index_bufs(kb2e_ctx* c) {
    return {{&c->keys, &c->sh_keys}, {&c->keys_sorted, &c->sh_keys_sorted}, {&c->sort_tmp, &c->sh_sort_tmp},
            {&c->flags, &c->sh_flags}, {&c->idx, &c->sh_idx}, {&c->seg_start, &c->sh_seg_start},
            {&c->nseg, &c->sh_nseg}, {&c->nvalid, &c->sh_nvalid}, {&c->batch_seg, &c->sh_batch_seg},
            {&c->ev_slot_sorted, &c->sh_ev_slot_sorted}, {&c->ev_inv, &c->sh_ev_inv}, {&c->seg_row, &c->sh_seg_row},
            {&c->rpar_ntiles, &c->sh_rpar_ntiles}, {&c->rpar_rel_begin, &c->sh_rpar_rel_begin},
            {&c->rpar_tile_first, &c->sh_rpar_tile_first}, {&c->rpar_tiles, &c->sh_rpar_tiles},
            {&c->rpar_batch_t0, &c->sh_rpar_batch_t0}, {&c->rpar_td_r, &c->sh_rpar_td_r},
            {&c->rpar_td_cnt, &c->sh_rpar_td_cnt}, {&c->rpar_td_kk, &c->sh_rpar_td_kk},
            {&c->rpar_td_ent, &c->sh_rpar_td_ent}, {&c->rpar_brel, &c->sh_rpar_brel},
            {&c->rpar_bnrel, &c->sh_rpar_bnrel},

            {&c->par_long_list, &c->sh_par_long_list}, {&c->par_long_count, &c->sh_par_long_count}};
}

void swap_index(kb2e_ctx* c) {
    for (auto& pr : index_bufs(c)) {
        std::swap(pr.first->p, pr.second->p);
        std::swap(pr.first->bytes, pr.second->bytes);
    }
    std::swap(c->pin_bnrel, c->pin_sh_bnrel);
}

void alloc_shadow_index(kb2e_ctx* c) {
    for (auto& pr : index_bufs(c)) {
        pr.second->free();
        if (pr.first->p) pr.second->alloc(pr.first->bytes);
    }
    c->index_pre_gen = -2;
}

// The epoch index of sample-stream set `set`, on stream st (timed on the batches' stream).
void build_index(kb2e_ctx* c, hipStream_t st, int set) {
    const int64_t nkeys = c->S * c->slots;
    KeyArgs ka{};
    ka.heads = c->heads.as<int32_t>();
    ka.tails = c->tails.as<int32_t>();
    ka.rels = c->rels.as<int32_t>();
    ka.si = c->si_[set].as<int32_t>();
    ka.sj = c->sj_[set].as<int32_t>();
    ka.side = c->side_[set].as<uint8_t>();
    ka.owner = c->cfg.model == KB2E_TRANSE ? nullptr : c->owner.as<int32_t>();
    ka.nsamples = c->S;
    ka.B = (int32_t)c->B;
    ka.sub = c->sub;
    ka.Bs = (int32_t)c->Bs;
    ka.ne = c->cfg.num_entities;
    ka.kl = c->kl;
    ka.keys = c->keys.as<uint64_t>();
    const int grid = (int)((c->S + 255) / 256);
    auto build = [&] {
        if (c->cfg.model == KB2E_TRANSR)
            emit_keys_kernel<8, true><<<grid, 256, 0, st>>>(ka);
        else
            emit_keys_kernel<6, false><<<grid, 256, 0, st>>>(ka);
        HIPCHK(hipGetLastError());
        // Keys are emitted sample-major and, within one sample and row, in (u, roles)
        // order, so a stable radix sort on the [batch | row] bits alone gives the
        // full-key order (sentinels stay last: batch nb-1 is never all-ones).
        const int lo_bit = getenv("KB2E_SORT_FULLKEY") ? 0 : c->kl.row_shift();
        size_t tb = c->sort_tmp_bytes;
        if (c->parallel() && c->cfg.model != KB2E_TRANSR) {  // the sorted position of every emitted key, for
                                                              // phase A's event records (TransE / TransH)
            HIPCHK(hipcub::DeviceRadixSort::SortPairs(c->sort_tmp.p, tb, c->keys.as<uint64_t>(),
                                                      c->keys_sorted.as<uint64_t>(), c->ev_iota.as<int32_t>(),
                                                      c->ev_slot_sorted.as<int32_t>(), (int)nkeys, lo_bit,
                                                      c->kl.total_bits(), st));
            inverse_perm_kernel<<<(int)((nkeys + 255) / 256), 256, 0, st>>>(c->ev_slot_sorted.as<int32_t>(),
                                                                                  nkeys, c->ev_inv.as<int32_t>());
            HIPCHK(hipGetLastError());
        } else {
            HIPCHK(hipcub::DeviceRadixSort::SortKeys(c->sort_tmp.p, tb, c->keys.as<uint64_t>(),
                                                     c->keys_sorted.as<uint64_t>(), (int)nkeys, lo_bit,
                                                     c->kl.total_bits(), st));
        }
        const int g2 = (int)((nkeys + 255) / 256);
        seg_flags_kernel<<<g2, 256, 0, st>>>(c->keys_sorted.as<uint64_t>(), nkeys, c->kl,
                                                     c->flags.as<int32_t>(), c->nvalid.as<int32_t>());
        HIPCHK(hipGetLastError());
        tb = c->sort_tmp_bytes;
        HIPCHK(hipcub::DeviceScan::ExclusiveSum(c->sort_tmp.p, tb, c->flags.as<int32_t>(),
                                                c->idx.as<int32_t>(), (int)nkeys, st));
        seg_scatter_kernel<<<g2, 256, 0, st>>>(c->flags.as<int32_t>(), c->idx.as<int32_t>(), nkeys,
                                                       c->seg_start.as<int32_t>(), c->nseg.as<int32_t>(),
                                                       c->nvalid.as<int32_t>());
        HIPCHK(hipGetLastError());
        batch_begin_kernel<<<256, 256, 0, st>>>(c->keys_sorted.as<uint64_t>(), c->seg_start.as<int32_t>(),
                                                        c->nseg.as<int32_t>(), (int)c->nbi, c->kl,
                                                        c->batch_seg.as<int32_t>());
        HIPCHK(hipGetLastError());
        if (c->cfg.model != KB2E_TRANSE && !c->parallel()) build_owner_index(c);
        if (c->parallel()) {
            seg_rows_kernel<<<256, 256, 0, st>>>(c->keys_sorted.as<uint64_t>(), c->seg_start.as<int32_t>(),
                                                       c->nseg.as<int32_t>(), c->kl, c->seg_row.as<int32_t>());
            HIPCHK(hipGetLastError());
            if (c->cfg.model != KB2E_TRANSE) build_transr_tiles(c, c->cfg.model == KB2E_TRANSR, st, set);
        }
        if (c->cfg.model != KB2E_TRANSR && c->cfg.schedule == KB2E_SCHEDULE_PARALLEL && c->apply_long_min > 0) {
            long_lists_kernel<<<(int)c->nb, 1024, 0, st>>>(
                c->seg_start.as<int32_t>(), c->batch_seg.as<int32_t>(), c->apply_long_min, c->par_long_cap,
                c->par_long_list.as<int32_t>(), c->par_long_count.as<int32_t>());
            HIPCHK(hipGetLastError());
        }
    };
    if (st == c->stream) c->timed("index", build);
    else build();
}

// ----------------------------------------------------------------- sampling

void upload_stream(kb2e_ctx* c, int set, hipStream_t st) {
    HIPCHK(hipMemcpyAsync(c->si_[set].p, c->pin_si, c->S * sizeof(int32_t), hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(c->sj_[set].p, c->pin_sj, c->S * sizeof(int32_t), hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(c->side_[set].p, c->pin_side, c->S, hipMemcpyHostToDevice, st));
}

// `doubling`: pointer doubling's K = log S levels of next[] (the fallback); the
// chunked chain reads only next[] itself (K5: 24 levels were 7.9 GB)
void ensure_sampler_capacity(kb2e_ctx* c, int64_t nraw, bool doubling) {
    const int K = doubling ? std::max(1, bits_for(std::max<int64_t>(c->S - 1, 1))) : 1;
    if (nraw <= c->nraw_cap && K <= c->levels_cap) return;
    c->words.alloc(nraw * 4);
    c->levels.alloc((size_t)K * (nraw + 1) * 4);
    c->levels_cap = K;
    c->jfin.alloc(nraw * 4);
    c->sidefin.alloc(nraw);
    c->raw_words.alloc((nraw + GlibcRand::kDeg) * 4);
    c->glibc_starts.alloc(((nraw + kGlibcBlock - 1) / kGlibcBlock) * GlibcRand::kDeg * 4);
    const int64_t nchunks = (nraw + kChainW - 1) / kChainW, nsuper = (nchunks + kChainG - 1) / kChainG;
    c->chain_table.alloc((size_t)nchunks * 64 * 4);
    c->chain_super.alloc((size_t)nsuper * 64 * 8);
    c->chain_sc.alloc((size_t)nsuper * 8);
    c->chain_ch.alloc((size_t)nchunks * 8);
    c->chain_overflow.alloc(16);
    c->nraw_cap = nraw;
}

// The glibc jump table (glibc_rand.hpp) on the device, made once per context.
void ensure_jump_table(kb2e_ctx* c) {
    if (c->glibc_table.p) return;
    std::vector<uint32_t> C((size_t)GlibcRand::kDeg * kGlibcBlock);
    glibc_jump_table(kGlibcBlock, C.data());
    c->glibc_table.alloc(C.size() * 4);
    HIPCHK(hipMemcpy(c->glibc_table.p, C.data(), C.size() * 4, hipMemcpyHostToDevice));
    // M (the window after kGlibcBlock words from the window before) and its squares
    constexpr int D = GlibcRand::kDeg;
    std::vector<uint32_t> P((size_t)kGlibcPowLevels * D * D);
    for (int j = 0; j < D; ++j)
        for (int m = 0; m < D; ++m) P[(size_t)j * D + m] = C[(size_t)m * kGlibcBlock + (kGlibcBlock - D + j)];
    for (int k = 1; k < kGlibcPowLevels; ++k) {
        const uint32_t* A = P.data() + (size_t)(k - 1) * D * D;
        uint32_t* Q = P.data() + (size_t)k * D * D;
        for (int i = 0; i < D; ++i)
            for (int j = 0; j < D; ++j) {
                uint32_t v = 0;
                for (int m = 0; m < D; ++m) v += A[i * D + m] * A[m * D + j];
                Q[i * D + j] = v;
            }
    }
    c->glibc_pow.alloc(P.size() * 4);
    HIPCHK(hipMemcpy(c->glibc_pow.p, P.data(), P.size() * 4, hipMemcpyHostToDevice));
}

// Draw the stream of the epoch that follows the committed rng state into set
// cur^1, on the side stream: the device makes the epoch's raw glibc words from
// the generator's 31-word window (jump table, kernels_sampler.hpp) and resolves
// the rejection chain.  Nothing is committed until start_epoch consumes it.
void launch_prefetch(kb2e_ctx* c) {
    const int set = c->cur ^ 1;
    const int64_t nraw = (int64_t)(c->words_per_sample * c->S) + 4096;
    const bool doubling = c->sampler_doubling || getenv("KB2E_SAMPLER_DOUBLING");
    ensure_sampler_capacity(c, nraw, doubling);
    c->nraw = nraw;
    ensure_jump_table(c);
    GlibcWindow win;
    c->rng.window(win.w);
    hipStream_t st = c->side_stream;
    // set cur^1 may still be read by the epoch before the current one
    HIPCHK(hipStreamWaitEvent(st, c->ev_epoch_done, 0));
    {
        const int64_t nblocks = (nraw + kGlibcBlock - 1) / kGlibcBlock;
        if (nblocks >= (int64_t)1 << kGlibcPowLevels) throw std::runtime_error("sampler word buffer too large");
        glibc_starts_pow_kernel<<<(int)nblocks, 64, 0, st>>>(win, c->glibc_pow.as<uint32_t>(),
                                                             c->glibc_starts.as<uint32_t>(),
                                                             c->raw_words.as<uint32_t>(),
                                                             c->chain_overflow.as<int32_t>());
        HIPCHK(hipGetLastError());
        glibc_words_kernel<<<(int)((nraw + 255) / 256), 256, 0, st>>>(
            c->glibc_table.as<uint32_t>(), kGlibcBlock, c->glibc_starts.as<uint32_t>(), nraw,
            c->raw_words.as<uint32_t>(), c->words.as<int32_t>());
        HIPCHK(hipGetLastError());
    }
    const int K = std::max(1, bits_for(std::max<int64_t>(c->S - 1, 1)));
    SamplerArgs a{};
    a.words = c->words.as<int32_t>();
    a.nraw = nraw;
    a.trip = c->trip_eb ? nullptr : c->trip.as<int4>();
    a.trip8 = c->trip_eb ? c->trip.as<uint64_t>() : nullptr;
    a.eb = c->trip_eb;
    a.rb = c->trip_rb;
    a.ntrain = (int32_t)c->ts.size();
    a.ne = c->cfg.num_entities;
    a.slots = c->filter_slots.as<uint64_t>();
    a.mask = c->ts.filter.mask;
    a.bloom = c->filter_bloom.as<uint64_t>();
    a.bloom_mask = c->ts.filter.bloom_mask;
    a.nr64 = (uint64_t)c->cfg.num_relations;
    a.ne64 = (uint64_t)c->cfg.num_entities;
    a.next = c->levels.as<int32_t>();
    a.jfin = c->jfin.as<int32_t>();
    a.sidefin = c->sidefin.as<uint8_t>();
    const int64_t stride = nraw + 1;
    auto launch = [&] {
        const char* sg = getenv("KB2E_SAMPLE_GRID");
        const int64_t g_full = (stride + 255) / 256;
        sample_len_kernel<<<(int)(sg ? std::max<int64_t>(1, std::min<int64_t>(g_full, atoi(sg))) : g_full), 256, 0,
                            st>>>(a);
        HIPCHK(hipGetLastError());
        if (!doubling) {
            ChunkArgs ch{};
            ch.next = a.next;
            ch.nraw = nraw;
            ch.nchunks = (int32_t)((nraw + kChainW - 1) / kChainW);
            ch.nsuper = (ch.nchunks + kChainG - 1) / kChainG;
            const char* em = getenv("KB2E_SAMPLER_EMAX");  // tests: a low limit forces the overflow path
            ch.emax = em ? std::max(1, std::min(kChainEmax, atoi(em))) : kChainEmax;
            ch.table = c->chain_table.as<uint32_t>();
            ch.super = c->chain_super.as<uint2>();
            ch.sc_state = c->chain_sc.as<uint2>();
            ch.ch_state = c->chain_ch.as<uint2>();
            ch.overflow = c->chain_overflow.as<int32_t>();
            ch.nsamples = c->S;
            ch.words = a.words;
            ch.jfin = a.jfin;
            ch.sidefin = a.sidefin;
            ch.ntrain = a.ntrain;
            ch.si = c->si_[set].as<int32_t>();
            ch.sj = c->sj_[set].as<int32_t>();
            ch.side = c->side_[set].as<uint8_t>();
            ch.consumed = c->consumed_dev.as<int64_t>();
            chain_table_kernel<<<ch.nchunks, 64, 0, st>>>(ch);
            chain_super_kernel<<<ch.nsuper, 64, 0, st>>>(ch);
            chain_top_kernel<<<1, 64, 0, st>>>(ch);
            chain_entries_kernel<<<ch.nsuper, 64, 0, st>>>(ch);
            chain_emit_kernel<<<ch.nchunks, 256, 0, st>>>(ch);
            HIPCHK(hipGetLastError());
            return;
        }
        for (int k = 1; k < K; ++k) {
            sample_double_kernel<<<(int)((stride + 255) / 256), 256, 0, st>>>(
                c->levels.as<int32_t>() + (int64_t)(k - 1) * stride, c->levels.as<int32_t>() + (int64_t)k * stride,
                stride);
            HIPCHK(hipGetLastError());
        }
        ChainArgs ca{};
        ca.levels = c->levels.as<int32_t>();
        ca.K = K;
        ca.stride = stride;
        ca.nsamples = c->S;
        ca.nraw = nraw;
        ca.words = a.words;
        ca.jfin = a.jfin;
        ca.sidefin = a.sidefin;
        ca.next = a.next;
        ca.ntrain = a.ntrain;
        ca.si = c->si_[set].as<int32_t>();
        ca.sj = c->sj_[set].as<int32_t>();
        ca.side = c->side_[set].as<uint8_t>();
        ca.consumed = c->consumed_dev.as<int64_t>();
        sample_chain_kernel<<<(int)((c->S + 255) / 256), 256, 0, st>>>(ca);
        HIPCHK(hipGetLastError());
    };
    if (c->prof) {
        hipEvent_t e0 = c->get_event(), e1 = c->get_event();
        HIPCHK(hipEventRecord(e0, st));
        launch();
        HIPCHK(hipEventRecord(e1, st));
        c->pending.push_back({"sample", e0, e1});
    } else {
        launch();
    }
    glibc_window_kernel<<<1, 64, 0, st>>>(c->raw_words.as<uint32_t>(), c->consumed_dev.as<int64_t>(),
                                          c->win_dev.as<uint32_t>());
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(c->pin_consumed, c->consumed_dev.p, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(c->pin_win, c->win_dev.p, GlibcRand::kDeg * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipEventRecord(c->ev_sampled, st));
    c->prefetch_valid = true;
    c->prefetch_version = c->rng_version;
    c->prefetch_gen++;
}

// Make set `cur` hold this epoch's stream and commit the rng past it.
void start_epoch_stream(kb2e_ctx* c) {
    if (c->cfg.sampler == KB2E_SAMPLER_REPLAY || c->host_sampler) {
        if (c->cfg.sampler == KB2E_SAMPLER_REPLAY) {
            if (c->rp_pos + c->S > (int64_t)c->rp_si.size())
                throw std::invalid_argument("replay stream exhausted: supply a full epoch of samples");
            std::memcpy(c->pin_si, c->rp_si.data() + c->rp_pos, c->S * sizeof(int32_t));
            std::memcpy(c->pin_sj, c->rp_sj.data() + c->rp_pos, c->S * sizeof(int32_t));
            std::memcpy(c->pin_side, c->rp_side.data() + c->rp_pos, c->S);
            c->rp_pos += c->S;
        } else {
            for (int64_t k = 0; k < c->S; ++k)
                if (!HostSampler::draw(c->rng, c->ts, c->cfg.method, c->pin_si[k], c->pin_sj[k], c->pin_side[k]))
                    throw std::runtime_error("negative sampler cannot terminate: every entity completes a training triple");
            c->rng_version++;
        }
        // the previous epoch may still read set cur: use the other set
        c->committed_gen = -1;
        c->cur ^= 1;
        upload_stream(c, c->cur, c->stream);
        HIPCHK(hipStreamSynchronize(c->stream));  // pinned buffers are reused next epoch
        return;
    }
    for (int attempt = 0;; ++attempt) {
        if (!c->prefetch_valid || c->prefetch_version != c->rng_version) launch_prefetch(c);
        HIPCHK(hipEventSynchronize(c->ev_sampled));
        const int64_t used = *c->pin_consumed;
        if (used == -2) {  // a sample longer than the chunked chain tabulates: redraw by doubling
            c->sampler_doubling = true;
            c->prefetch_valid = false;
            continue;
        }
        if (used >= 0) {
            c->rng.set_window(c->pin_win);  // the generator after the epoch's `used` words
            c->rng_version++;
            // the next epoch speculates on 3% (+ 4096) more words than this one used: every
            // word position costs sample_len a triple gather and a filter probe
            c->words_per_sample = 1.03 * (double)used / (double)c->S;
            break;
        }
        // the speculative word buffer ran out (long rejection runs): retry larger
        c->prefetch_valid = false;
        c->words_per_sample *= 1.5;
        if (attempt > 20)
            throw std::runtime_error("negative sampler cannot terminate: every entity completes a training triple");
    }
    c->prefetch_valid = false;
    c->committed_gen = c->prefetch_gen;  // the prefetch this epoch consumes
    c->cur ^= 1;
    HIPCHK(hipStreamWaitEvent(c->stream, c->ev_sampled, 0));
    // The next epoch's stream is drawn beside this epoch's batches (launch_next,
    // once the epoch's first batch is queued): it writes the set the previous
    // epoch read (the side stream waits for that epoch's end marker) and its rng
    // start is this epoch's committed end.
    c->next_pending = true;
}

// The next epoch's sample stream and (PARALLEL) its event index, on the side stream.
void launch_next(kb2e_ctx* c) {
    c->next_pending = false;
    launch_prefetch(c);
    if (c->parallel() && c->sh_keys.p) {
        // into the shadow index buffers (the set the previous epoch read, which the
        // prefetch already waited for), right after the sample stream
        swap_index(c);
        build_index(c, c->side_stream, c->cur ^ 1);
        swap_index(c);
        HIPCHK(hipEventRecord(c->ev_index, c->side_stream));
        c->index_pre_gen = c->prefetch_gen;
    }
}

// --------------------------------------------------------------- the batch

template <typename T>
ScoreArgs<T> score_args(kb2e_ctx* c, int64_t b) {
    ScoreArgs<T> a{};
    a.heads = c->heads.as<int32_t>();
    a.tails = c->tails.as<int32_t>();
    a.rels = c->rels.as<int32_t>();
    a.si = c->si() + b * c->B;
    a.sj = c->sj() + b * c->B;
    a.side = c->side() + b * c->B;
    a.B = (int32_t)c->B;
    a.n = c->n;
    a.ld = c->ld;
    a.nw = c->nw;
    a.ne = c->cfg.num_entities;
    a.ent = c->ent.as<T>();
    a.rel = c->rel.as<T>();
    a.w = c->w.as<T>();
    a.margin = c->cfg.margin;
    a.act = c->act.as<uint8_t>() + b * c->B;
    a.loss = c->loss.as<double>() + b * c->B;
    a.xbits = c->xbits.as<uint64_t>();
    a.xreal = c->xreal.as<T>();
    return a;
}

template <typename T, int CH>
void run_batch_transe(kb2e_ctx* c, int64_t b) {
    ScoreArgs<T> sa = score_args<T>(c, b);
    const bool l1 = c->cfg.distance == 0;
    const int grid = (int)((c->B + 3) / 4);
    c->timed("score", [&] {
        if (l1) transe_score_kernel<T, CH, true><<<grid, 256, 0, c->stream>>>(sa);
        else transe_score_kernel<T, CH, false><<<grid, 256, 0, c->stream>>>(sa);
        HIPCHK(hipGetLastError());
    });
    FoldArgs<T> fa{};
    fa.keys = c->keys_sorted.as<uint64_t>();
    fa.seg_start = c->seg_start.as<int32_t>();
    fa.batch_seg = c->batch_seg.as<int32_t>();
    fa.batch = (int32_t)b;
    fa.kl = c->kl;
    fa.ne = c->cfg.num_entities;
    fa.n = c->n;
    fa.ld = c->ld;
    fa.nw = c->nw;
    fa.ent = c->ent.as<T>();
    fa.rel = c->rel.as<T>();
    fa.lr = c->cfg.learning_rate;
    fa.act = sa.act;
    fa.xbits = sa.xbits;
    fa.xreal = sa.xreal;
    fa.gram_min = c->gram_min;
    const bool use_long = l1 && c->long_min > 0 && c->gram_min > 0;
    fa.long_min = use_long ? c->long_min : 0;
    // Enough waves for every touched row of a batch (<= 6 B segments).
    const int64_t max_seg = std::min<int64_t>(c->B * 6, (int64_t)c->cfg.num_entities + c->cfg.num_relations);
    const int fgrid = (int)std::max<int64_t>(1, std::min<int64_t>((max_seg + 3) / 4, 4096));
    hipEvent_t span = c->begin_span();  // phase B as a whole: both fold kernels and the join
    if (use_long) {
        // long segments: one 4-wave workgroup each, on the fold stream, beside the per-row fold
        long_segments_kernel<<<1, 1024, 0, c->stream>>>(fa.seg_start, fa.batch_seg, fa.batch, c->long_min,
                                                        c->long_list.as<int32_t>(), c->long_count.as<int32_t>());
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(c->ev_fold_a, c->stream));
        HIPCHK(hipStreamWaitEvent(c->fold_stream, c->ev_fold_a, 0));
        c->timed_on(c->fold_stream, "fold_long", [&] {
            transe_fold_long_kernel<T, CH><<<128, 256, fold_long_lds_bytes<T, CH>(), c->fold_stream>>>(
                fa, c->long_list.as<int32_t>(), c->long_count.as<int32_t>());
            HIPCHK(hipGetLastError());
        });
        HIPCHK(hipEventRecord(c->ev_fold_b, c->fold_stream));
    }
    c->timed("fold", [&] {
        if (l1) transe_fold_kernel<T, CH, true><<<fgrid, 256, 0, c->stream>>>(fa);
        else transe_fold_kernel<T, CH, false><<<fgrid, 256, 0, c->stream>>>(fa);
        HIPCHK(hipGetLastError());
    });
    if (use_long) HIPCHK(hipStreamWaitEvent(c->stream, c->ev_fold_b, 0));
    c->end_span("fold_phase", span);
}

EventRecs event_recs(kb2e_ctx* c) {
    EventRecs er{};
    er.meta = c->ev_meta.as<int32_t>();
    er.words = c->ev_words.as<uint64_t>();
    er.inv = c->ev_inv.as<int32_t>();
    er.keys = c->keys.as<uint64_t>();
    er.seg_row = c->seg_row.as<int32_t>();
    er.slots = c->slots;
    return er;
}

// PARALLEL schedule (kernels_parallel.hpp): the same phase A, then every
// touched row gets its summed delta and one norm.  Long segments (the hot
// relations and entities) take a 16-wave workgroup each.
template <typename T, int CH>
void run_batch_transe_parallel(kb2e_ctx* c, int64_t b) {
    ScoreArgs<T> sa = score_args<T>(c, b);
    const bool l1 = c->cfg.distance == 0;
    const int grid = (int)((c->B + 3) / 4);
    const EventRecs er = event_recs(c);
    hipEvent_t e0, e1;
    c->ev_begin("score", e0);
    c->ev_end(e1);
    if (l1) c->launch(transe_score_kernel<T, CH, true, true>, dim3(grid), dim3(256), 0, e0, e1, sa, er, c->kl, b * c->B);
    else c->launch(transe_score_kernel<T, CH, false, true>, dim3(grid), dim3(256), 0, e0, e1, sa, er, c->kl, b * c->B);
    FoldArgs<T> fa{};
    fa.keys = c->keys_sorted.as<uint64_t>();
    fa.seg_start = c->seg_start.as<int32_t>();
    fa.batch_seg = c->batch_seg.as<int32_t>();
    fa.batch = (int32_t)b;
    fa.kl = c->kl;
    fa.ne = c->cfg.num_entities;
    fa.n = c->n;
    fa.ld = c->ld;
    fa.nw = c->nw;
    fa.ent = c->ent.as<T>();
    fa.rel = c->rel.as<T>();
    fa.lr = c->cfg.learning_rate;
    fa.act = sa.act;
    fa.xbits = sa.xbits;
    fa.xreal = sa.xreal;
    fa.gram_min = 0;
    fa.long_min = c->apply_long_min;
    // phase B is this one kernel
    c->ev_begin("apply", e0);
    c->ev_end(e1);
    const int32_t* ll = c->par_long_list.as<int32_t>();
    const int32_t* lc = c->par_long_count.as<int32_t>();
    if (l1)
        c->launch(transe_apply_kernel<T, CH, true>, dim3(c->apply_grid), dim3(1024), 0, e0, e1, fa, er, ll, lc,
                  c->par_long_cap);
    else
        c->launch(transe_apply_kernel<T, CH, false>, dim3(c->apply_grid), dim3(1024), 0, e0, e1, fa, er, ll, lc,
                  c->par_long_cap);
    if (c->pending.size() > 4096) c->flush_timers();
}

template <typename K>
void allow_lds(K kernel, size_t bytes) {
    (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

void prepare_fold_long_kernels() {
    allow_lds(transe_fold_long_kernel<double, 1>, fold_long_lds_bytes<double, 1>());
    allow_lds(transe_fold_long_kernel<double, 2>, fold_long_lds_bytes<double, 2>());
    allow_lds(transe_fold_long_kernel<double, 4>, fold_long_lds_bytes<double, 4>());
    allow_lds(transe_fold_long_kernel<float, 1>, fold_long_lds_bytes<float, 1>());
    allow_lds(transe_fold_long_kernel<float, 2>, fold_long_lds_bytes<float, 2>());
    allow_lds(transe_fold_long_kernel<float, 4>, fold_long_lds_bytes<float, 4>());
}

template <typename T>
void run_batch(kb2e_ctx* c, int64_t b) {
    if (c->cfg.model == KB2E_TRANSE && c->cfg.schedule == KB2E_SCHEDULE_PARALLEL) {
        switch (c->ch) {
            case 1: run_batch_transe_parallel<T, 1>(c, b); break;
            case 2: run_batch_transe_parallel<T, 2>(c, b); break;
            default: run_batch_transe_parallel<T, 4>(c, b); break;
        }
    } else if (c->cfg.model == KB2E_TRANSE) {
        switch (c->ch) {
            case 1: run_batch_transe<T, 1>(c, b); break;
            case 2: run_batch_transe<T, 2>(c, b); break;
            default: run_batch_transe<T, 4>(c, b); break;
        }
    } else if (c->cfg.model == KB2E_TRANSR && c->parallel()) {
        run_batch_transr_parallel<T>(c, b);
    } else if (c->cfg.model == KB2E_TRANSH && c->parallel()) {
        switch (c->ch) {
            case 1: run_batch_transh_parallel<T, 1>(c, b); break;
            case 2: run_batch_transh_parallel<T, 2>(c, b); break;
            default: run_batch_transh_parallel<T, 4>(c, b); break;
        }
    } else {
        run_batch_relowner<T>(c, b);
    }
}

// Epoch statistics (loss, hinge-active count) summed on the device without a
// host round trip: 256 fixed slices summed by one block each, then the slices
// in order by one block into the running accumulator.  Deterministic.
constexpr int kStatSlices = 256;

__global__ __launch_bounds__(256) void stats_partial_kernel(const double* loss, const uint8_t* act, int64_t lo,
                                                            int64_t hi, double* part) {
    __shared__ double sl[256], sa[256];
    const int64_t n = hi - lo;
    const int64_t b0 = lo + n * blockIdx.x / kStatSlices, b1 = lo + n * (blockIdx.x + 1) / kStatSlices;
    double l = 0, a = 0;
    for (int64_t k = b0 + threadIdx.x; k < b1; k += blockDim.x) {
        l += loss[k];
        a += act[k];
    }
    sl[threadIdx.x] = l;
    sa[threadIdx.x] = a;
    __syncthreads();
    for (int s = blockDim.x / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) {
            sl[threadIdx.x] += sl[threadIdx.x + s];
            sa[threadIdx.x] += sa[threadIdx.x + s];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        part[2 * blockIdx.x] = sl[0];
        part[2 * blockIdx.x + 1] = sa[0];
    }
}

__global__ __launch_bounds__(256) void stats_final_kernel(const double* part, double* acc) {
    __shared__ double sl[kStatSlices], sa[kStatSlices];
    sl[threadIdx.x] = part[2 * threadIdx.x];
    sa[threadIdx.x] = part[2 * threadIdx.x + 1];
    __syncthreads();
    for (int s = kStatSlices / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) {
            sl[threadIdx.x] += sl[threadIdx.x + s];
            sa[threadIdx.x] += sa[threadIdx.x + s];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        acc[0] += sl[0];
        acc[1] += sa[0];
    }
}

// Queue the sums of samples [reduced_upto, upto) of the current epoch into the
// device accumulator (asynchronous).
void reduce_stats(kb2e_ctx* c, int64_t upto) {
    if (upto <= c->reduced_upto) return;
    double* part = c->stats.as<double>() + 2;
    stats_partial_kernel<<<kStatSlices, 256, 0, c->stream>>>(c->loss.as<double>(), c->act.as<uint8_t>(),
                                                               c->reduced_upto, upto, part);
    HIPCHK(hipGetLastError());
    stats_final_kernel<<<1, kStatSlices, 0, c->stream>>>(part, c->stats.as<double>());
    HIPCHK(hipGetLastError());
    c->reduced_upto = upto;
}

// Move the device accumulator into the host totals (synchronises the stream).
void collect_stats(kb2e_ctx* c) {
    double h[2];
    HIPCHK(hipMemcpyAsync(h, c->stats.p, sizeof(h), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemsetAsync(c->stats.p, 0, sizeof(h), c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->acc_loss += h[0];
    c->acc_active += (int64_t)llround(h[1]);
    check_dataflow(c);
}

void run_batches(kb2e_ctx* c, int64_t count) {
    if (!c->have_triples || !c->have_params) throw std::logic_error("upload triples and params first");
    for (int64_t q = 0; q < count; ++q) {
        if (c->epoch_pos == 0 && !c->epoch_ready) {
            start_epoch_stream(c);
            // (PARALLEL TransR: the chain launches' grids, the batches' relation counts, come
            // to the host with the index)
            const bool counts = c->rpar_bnrel.p != nullptr;
            if (c->committed_gen >= 0 && c->index_pre_gen == c->committed_gen) {
                HIPCHK(hipStreamWaitEvent(c->stream, c->ev_index, 0));  // built beside the previous epoch
                if (counts) HIPCHK(hipEventSynchronize(c->ev_index));  // (long done: built an epoch ahead)
                swap_index(c);
            } else {
                build_index(c, c->stream, c->cur);
                if (counts) HIPCHK(hipStreamSynchronize(c->stream));
            }
            c->epoch_ready = true;
            c->reduced_upto = 0;
        }
        c->prof_batch = (c->prof_counter++ % c->prof_period) == 0;
        if (c->f64()) run_batch<double>(c, c->epoch_pos);
        else run_batch<float>(c, c->epoch_pos);
        c->prof_batch = true;
        if (++c->epoch_pos == c->nb) {
            // Overlap the next epoch's sampling with this epoch's batches.  It
            // writes the set the previous epoch read, so it waits for the
            // previous epoch's end marker (recorded below for the next one).
            HIPCHK(hipEventRecord(c->ev_epoch_done, c->stream));
            reduce_stats(c, c->S);
            c->epoch_pos = 0;
            c->epoch_ready = false;
        }
        // after the epoch's first batch is queued: the GPU runs it while the host
        // queues the side stream's work
        if (c->next_pending) launch_next(c);
    }
}

void setup_buffers(kb2e_ctx* c) {
    const kb2e_config& g = c->cfg;
    c->esize = c->f64() ? 8 : 4;
    c->n = g.dim;
    c->ld = (g.dim + 1) & ~1;
    c->ch = (g.dim + kWave * kVec - 1) / (kWave * kVec);
    c->nw = c->ch * kVec;
    const size_t es = (size_t)c->esize;
    c->ent.alloc((size_t)g.num_entities * c->ld * es);
    c->rel.alloc((size_t)g.num_relations * c->ld * es);
    memset_sync(c->ent.p, 0, c->ent.bytes);
    memset_sync(c->rel.p, 0, c->rel.bytes);
    if (g.model == KB2E_TRANSH) c->w_elems = (int64_t)g.num_relations * g.dim;
    if (g.model == KB2E_TRANSR) c->w_elems = (int64_t)g.num_relations * g.dim * g.dim;
    c->w.alloc((size_t)std::max<int64_t>(1, w_rows(c)) * c->ld * es);
    memset_sync(c->w.p, 0, c->w.bytes);
    if (g.model == KB2E_TRANSR) {  // committed matrices (start-of-batch snapshot)
        c->wsnap.alloc(c->w.bytes);
        memset_sync(c->wsnap.p, 0, c->wsnap.bytes);
    }
}

void setup_epoch_buffers(kb2e_ctx* c) {
    const kb2e_config& g = c->cfg;
    const int64_t ntrain = c->ts.size();
    c->B = ntrain / g.num_batches;
    c->nb = g.num_batches;
    c->S = c->B * c->nb;
    if (c->B < 1) throw std::invalid_argument("fewer training triples than batches");
    // PARALLEL TransR sub-batches: the event index cuts every batch into `sub` index
    // batches of Bs samples (the last one the rest), each one phase B of its own
    c->sub = 1;
    c->Bs = c->B;
    if (g.model == KB2E_TRANSR && g.schedule == KB2E_SCHEDULE_PARALLEL && g.sub_batches > 1) {
        c->Bs = (c->B + g.sub_batches - 1) / g.sub_batches;
        c->sub = (int32_t)((c->B + c->Bs - 1) / c->Bs);  // (the non-empty ones)
    }
    c->nbi = c->nb * c->sub;
    c->long_list.alloc((size_t)c->B * c->slots * 4);
    c->long_count.alloc(16);
    for (int q = 0; q < 2; ++q) {
        c->si_[q].alloc(c->S * 4);
        c->sj_[q].alloc(c->S * 4);
        c->side_[q].alloc(c->S);
    }
    c->prefetch_valid = false;
    c->next_pending = false;
    c->nraw_cap = 0;
    c->levels_cap = 0;
    c->consumed_dev.alloc(16);
    if (!c->pin_consumed) HIPCHK(hipHostMalloc((void**)&c->pin_consumed, 16, 0));
    if (!c->pin_win) HIPCHK(hipHostMalloc((void**)&c->pin_win, 32 * 4, 0));
    c->win_dev.alloc(32 * 4);
    if (c->pin_si) { (void)hipHostFree(c->pin_si); (void)hipHostFree(c->pin_sj); (void)hipHostFree(c->pin_side); }
    HIPCHK(hipHostMalloc((void**)&c->pin_si, c->S * 4, 0));
    HIPCHK(hipHostMalloc((void**)&c->pin_sj, c->S * 4, 0));
    HIPCHK(hipHostMalloc((void**)&c->pin_side, c->S, 0));
    // keys
    c->slots = g.model == KB2E_TRANSR ? 8 : 6;
    const int64_t nowners = g.model == KB2E_TRANSE ? g.num_relations : c->plan.num_owners;
    c->kl.kk_bits = bits_for(c->B);
    c->kl.row_bits = bits_for((int64_t)g.num_entities + nowners);
    c->kl.batch_bits = bits_for(c->nbi);  // holds nbi, so index batch nbi-1 is never all-ones
    if (c->kl.total_bits() > 64) throw std::invalid_argument("problem too large for 64-bit event keys");
    const int64_t nkeys = c->S * c->slots;
    if (nkeys >= (1ll << 31)) throw std::invalid_argument("epoch too large for one index (> 2^31 events)");
    c->keys.alloc(nkeys * 8);
    c->keys_sorted.alloc(nkeys * 8);
    c->flags.alloc(nkeys * 4);
    c->idx.alloc(nkeys * 4);
    c->seg_start.alloc((nkeys + 1) * 4);
    c->nseg.alloc(16);
    c->nvalid.alloc(16);
    c->batch_seg.alloc((c->nbi + 1) * 4);
    size_t t1 = 0, t2 = 0, t3 = 0;
    HIPCHK(hipcub::DeviceRadixSort::SortKeys(nullptr, t1, (uint64_t*)nullptr, (uint64_t*)nullptr, (int)nkeys, 0,
                                             c->kl.total_bits(), c->stream));
    if (c->parallel()) {
        HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, t3, (uint64_t*)nullptr, (uint64_t*)nullptr,
                                                  (int32_t*)nullptr, (int32_t*)nullptr, (int)nkeys, 0,
                                                  c->kl.total_bits(), c->stream));
        c->ev_iota.alloc(nkeys * 4);
        std::vector<int32_t> iota((size_t)nkeys);
        for (int64_t q = 0; q < nkeys; ++q) iota[q] = (int32_t)q;
        HIPCHK(hipMemcpy(c->ev_iota.p, iota.data(), nkeys * 4, hipMemcpyHostToDevice));
        c->ev_slot_sorted.alloc(nkeys * 4);
        c->ev_inv.alloc(nkeys * 4);
        c->seg_row.alloc((nkeys + 1) * 4);
        c->ev_meta.alloc(nkeys * 4);
        c->ev_words.alloc((size_t)nkeys * c->nw * 8);
    }
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, t2, (int32_t*)nullptr, (int32_t*)nullptr, (int)nkeys,
                                            c->stream));
    c->sort_tmp_bytes = std::max(std::max(t1, t2), t3);
    c->sort_tmp.alloc(c->sort_tmp_bytes);
    c->act.alloc(c->S);
    c->loss.alloc(c->S * 8);
    c->xbits.alloc((size_t)c->B * 2 * c->nw * 8);
    if (g.distance != 0 || g.model == KB2E_TRANSR)
        c->xreal.alloc((size_t)c->B * 2 * c->ld * c->esize);
    c->stats.alloc((2 + 2 * kStatSlices) * 8);
    memset_sync(c->stats.p, 0, c->stats.bytes);
    if (g.model != KB2E_TRANSR && g.schedule == KB2E_SCHEDULE_PARALLEL) {
        const int64_t per_batch = c->B * c->slots;
        c->par_long_cap = (int32_t)(c->apply_long_min > 0 ? std::min<int64_t>(per_batch, per_batch / c->apply_long_min + 1)
                                                         : 1);
        c->par_long_list.alloc((size_t)c->nb * c->par_long_cap * 4);
        c->par_long_count.alloc((size_t)c->nb * 4);
        // one 16-wave workgroup per CU, and at least one per long segment
        c->apply_grid = std::max(2 * c->num_cus, std::min<int>(c->par_long_cap, 4096));
        if (const char* ag = getenv("KB2E_APPLY_GRID")) c->apply_grid = std::max(1, atoi(ag));
    }
    setup_relowner_buffers(c);
    if (g.model == KB2E_TRANSR && g.schedule == KB2E_SCHEDULE_PARALLEL) setup_transr_parallel(c);
    if (g.model == KB2E_TRANSH && g.schedule == KB2E_SCHEDULE_PARALLEL) {
        c->hpar_orth.alloc((size_t)((c->B + 511) / 512) * 512);  // whole 8-byte words past B stay zero
        memset_sync(c->hpar_orth.p, 0, c->hpar_orth.bytes);
        c->hpar_ids.alloc((size_t)c->B * 8 * 4);  // (written for the flagged samples before they are read)
        c->hpar_count.alloc(3 * 4);  // (+ the batches whose relation pass ran: kb2e_counter)
        memset_sync(c->hpar_count.p, 0, c->hpar_count.bytes);
        const char* om = getenv("KB2E_HPAR_ORTH_MIN");  // tests: 0 always, a large value never
        c->hpar_orth_min = om ? (uint32_t)std::max(0, atoi(om)) : kOrthRelMin;
        const char* oq = getenv("KB2E_HPAR_ORTH_Q");  // tests: 0 lists the second sweep's flags again
        c->hpar_orth_q = oq ? std::max(0, std::min(kOrthQ, atoi(oq))) : kOrthQ;
        c->hpar_tag.alloc((size_t)c->cfg.num_entities * 8);  // zeroed: stamp 0 is never a batch's
        c->rpar_St = 1 << 30;  // build_transr_tiles(c, false): relation segment ranges only
        c->rpar_ntiles.alloc((size_t)(nkeys + 1) * 4);
        c->rpar_rel_begin.alloc((size_t)c->nb * 4);
    }
    if (c->parallel() && !getenv("KB2E_NO_PREINDEX")) alloc_shadow_index(c);  // the prebuilt next-epoch index
}

}  // namespace

#include "engine_relowner.inc"
#include "engine_transr_parallel.inc"
#include "engine_transh_parallel.inc"

namespace {
template <typename T, int CH>
__global__ __launch_bounds__(256) void renorm_kernel(T* table, int64_t rows, int ld, int n, const uint8_t* mask,
                                                     int div, bool ignore_short) {
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t r = wave; r < rows; r += nwaves) {
        if (mask && !mask[r / div]) continue;
        RowReg<T, CH> v;
        v.load(table + r * ld, n);
        v.norm(n, ignore_short);
        v.store(table + r * ld, n);
    }
}
// The model's norm constraint on `count` units of a table from `first` (units:
// entities, relations, or relations of the weights table), rows flagged in the
// DEVICE mask (indexed from `first`; nullptr = all): TransE rows and TransH
// entity/relation rows shrink to length <= 1 (common/utils.cpp:70-77), TransH
// normals and TransR entity/relation/matrix rows are scaled to unit length
// (transh/trainer.cpp:52, transr/trainer.cpp:174-180).  Asynchronous.
void renorm_rows(kb2e_ctx* c, int table, int64_t first, int64_t count, const uint8_t* dmask) {
    if (count <= 0) return;
    const int model = c->cfg.model;
    const bool unit = model == KB2E_TRANSR || table == 2;
    DevBuf* t = table == 0 ? &c->ent : table == 1 ? &c->rel : &c->w;
    const int div = model == KB2E_TRANSR && table == 2 ? c->n : 1;  // TransR: n matrix rows per relation
    const int64_t rows = count * div;
    const int64_t off = first * div * c->ld;
    const int grid = (int)std::min<int64_t>((rows + 3) / 4, 65535);
    auto go = [&](auto tag, auto chtag) {
        using T = decltype(tag);
        constexpr int CH = decltype(chtag)::value;
        renorm_kernel<T, CH><<<grid, 256, 0, c->stream>>>(t->as<T>() + off, rows, c->ld, c->n, dmask, div, !unit);
    };
    if (c->f64()) {
        if (c->ch == 1) go(double(), std::integral_constant<int, 1>());
        else if (c->ch == 2) go(double(), std::integral_constant<int, 2>());
        else go(double(), std::integral_constant<int, 4>());
    } else {
        if (c->ch == 1) go(float(), std::integral_constant<int, 1>());
        else if (c->ch == 2) go(float(), std::integral_constant<int, 2>());
        else go(float(), std::integral_constant<int, 4>());
    }
    HIPCHK(hipGetLastError());
}
}  // namespace

// ================================================================== C ABI

extern "C" {

void kb2e_default_config(kb2e_config* cfg) {
    if (!cfg) return;
    std::memset(cfg, 0, sizeof(*cfg));
    cfg->model = KB2E_TRANSE;
    cfg->dim = 100;              // DEFAULT_EMBEDDING_SIZE
    cfg->learning_rate = 0.001;  // DEFAULT_LEARNING_RATE
    cfg->margin = 1.0;           // DEFAULT_MARGIN
    cfg->method = 1;             // DEFAULT_METHOD = bern
    cfg->distance = 0;           // DEFAULT_DISTANCE = L1
    cfg->num_batches = 100;      // DEFAULT_NUM_BATCHES
    cfg->seed = 0;
    cfg->precision = 64;
    cfg->sampler = KB2E_SAMPLER_GLIBC;
    cfg->transr_compat = 1;
    cfg->device = 0;
    cfg->schedule = KB2E_SCHEDULE_ORDERED;
    cfg->sub_batches = 0;  // by width (default_sub_batches)
}

namespace {
// PARALLEL TransR sub-batches when kb2e_config.sub_batches is 0: the smallest count
// whose paired loss interval against the reference's seed envelope covers 0 at the
// widths measured (FB15k-shaped, compat, 100 batches, 5 seeds):
// n = 50 -> 2 (k = 1: -2.8 % [-4.3, -1.4]; k = 2: -0.8 % [-2.5, +0.9]), n = 100 -> 3
// (k = 2: -3.7 % [-5.4, -2.0]; k = 3: -1.8 % [-3.8, +0.1]); wider: 3 (unmeasured)
int32_t default_sub_batches(const kb2e_config& g) {
    if (g.model != KB2E_TRANSR || g.schedule != KB2E_SCHEDULE_PARALLEL) return 1;
    return g.dim <= 64 ? 2 : 3;
}
}  // namespace

kb2e_status kb2e_get_config(const kb2e_ctx* ctx, kb2e_config* out) {
    if (!ctx || !out) return KB2E_EINVAL;
    *out = ctx->cfg;
    return KB2E_OK;
}

kb2e_status kb2e_create(const kb2e_config* cfg, kb2e_ctx** out) {
    if (!cfg || !out) return KB2E_EINVAL;
    *out = nullptr;
    const kb2e_config& g = *cfg;
    if (g.model < 0 || g.model > 2 || g.dim < 1 || g.dim > 512 || g.num_entities < 1 || g.num_relations < 1 ||
        g.num_batches < 1 || (g.precision != 32 && g.precision != 64) || (g.method != 0 && g.method != 1) ||
        (g.distance != 0 && g.distance != 1) || (g.sampler != 0 && g.sampler != 1) ||
        (g.schedule != KB2E_SCHEDULE_ORDERED && g.schedule != KB2E_SCHEDULE_PARALLEL) || g.sub_batches < 0 ||
        g.sub_batches > 64)
        return KB2E_EINVAL;
    if (g.model == KB2E_TRANSR && g.num_relations > g.num_entities) return KB2E_EINVAL;
    std::unique_ptr<kb2e_ctx> c(new kb2e_ctx());
    c->cfg = g;
    if (c->cfg.sub_batches == 0) c->cfg.sub_batches = default_sub_batches(g);
    c->rng.seed_with(g.seed);
    kb2e_status s = guarded(c.get(), [&] {
        int ndev = 0;
        HIPCHK(hipGetDeviceCount(&ndev));
        if (g.device < 0 || g.device >= ndev) return fail(c.get(), KB2E_EDEVICE, "no such HIP device");
        HIPCHK(hipSetDevice(g.device));
        // the batches' streams high priority, the next epoch's sampling and index
        // (side stream) low: its workgroups fill what the batches leave idle
        int lo = 0, hi = 0;
        const char* sp = getenv("KB2E_STREAM_PRIO");
        if (!(sp && sp[0] == '0')) HIPCHK(hipDeviceGetStreamPriorityRange(&lo, &hi));
        HIPCHK(hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, hi));
        HIPCHK(hipStreamCreateWithPriority(&c->side_stream, hipStreamNonBlocking, lo));
        HIPCHK(hipStreamCreateWithPriority(&c->fold_stream, hipStreamNonBlocking, hi));
        HIPCHK(hipEventCreateWithFlags(&c->ev_fold_a, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&c->ev_fold_b, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&c->ev_sampled, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&c->ev_epoch_done, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&c->ev_index, hipEventDisableTiming));
        HIPCHK(hipEventRecord(c->ev_epoch_done, c->stream));
        HIPCHK(hipDeviceGetAttribute(&c->num_cus, hipDeviceAttributeMultiprocessorCount, g.device));
        prepare_relowner_kernels();
        prepare_fold_long_kernels();
        if (const char* gm = getenv("KB2E_GRAM_MIN")) c->gram_min = atoi(gm);
        if (const char* lm = getenv("KB2E_FOLD_LONG")) c->long_min = atoi(lm);
        if (const char* al = getenv("KB2E_APPLY_LONG")) c->apply_long_min = atoi(al);
        const char* hs = getenv("KB2E_HOST_SAMPLER");
        c->host_sampler = hs && hs[0] == '1';
        setup_buffers(c.get());
        HIPCHK(hipDeviceSynchronize());
        return KB2E_OK;
    });
    if (s != KB2E_OK) return s;
    *out = c.release();
    return KB2E_OK;
}

void kb2e_destroy(kb2e_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->cfg.device);
    delete ctx;
}

const char* kb2e_last_error(const kb2e_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

kb2e_status kb2e_upload_triples(kb2e_ctx* c, const int32_t* h, const int32_t* t, const int32_t* r, int64_t count) {
    return guarded(c, [&] {
        if (!h || !t || !r || count < 1) return fail(c, KB2E_EINVAL, "empty triple set");
        HIPCHK(hipSetDevice(c->cfg.device));
        c->ts.build(h, t, r, count, c->cfg.num_entities, c->cfg.num_relations);
        c->heads.alloc(count * 4);
        c->tails.alloc(count * 4);
        c->rels.alloc(count * 4);
        HIPCHK(hipMemcpy(c->heads.p, h, count * 4, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(c->tails.p, t, count * 4, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(c->rels.p, r, count * 4, hipMemcpyHostToDevice));
        c->filter_slots.alloc(c->ts.filter.slots.size() * 8);
        HIPCHK(hipMemcpy(c->filter_slots.p, c->ts.filter.slots.data(), c->ts.filter.slots.size() * 8,
                         hipMemcpyHostToDevice));
        c->filter_bloom.alloc(c->ts.filter.bloom.size() * 8);
        HIPCHK(hipMemcpy(c->filter_bloom.p, c->ts.filter.bloom.data(), c->ts.filter.bloom.size() * 8,
                         hipMemcpyHostToDevice));
        {  // relations by training frequency, most frequent first (the PARALLEL TransR chain
           // kernels start the hot relations' long chains first: kernels_transr_chainw.hpp)
            std::vector<int32_t> order((size_t)c->cfg.num_relations);
            for (int32_t q = 0; q < c->cfg.num_relations; ++q) order[q] = q;
            std::stable_sort(order.begin(), order.end(),
                             [&](int32_t x, int32_t y) { return c->ts.rel_count[x] > c->ts.rel_count[y]; });
            c->rel_order.alloc(order.size() * 4);
            HIPCHK(hipMemcpy(c->rel_order.p, order.data(), order.size() * 4, hipMemcpyHostToDevice));
        }
        std::vector<double> pr(c->ts.pr);
        if (c->cfg.method == 0) std::fill(pr.begin(), pr.end(), 500.0);  // common/trainer.cpp:84-86
        c->pr_dev.alloc(pr.size() * 8);
        HIPCHK(hipMemcpy(c->pr_dev.p, pr.data(), pr.size() * 8, hipMemcpyHostToDevice));
        {  // sample_len's packed triples: (double)(rand() % 1000) < pr[r] <=> rand() % 1000 < thr[r]
            std::vector<int32_t> thr(pr.size());
            for (size_t q = 0; q < pr.size(); ++q) {
                int32_t k = 0;
                while (k < 1000 && (double)k < pr[q]) ++k;
                thr[q] = k;
            }
            // 8 bytes a triple when two entity ids, a relation id and the threshold
            // (< 1024) fit (FB15k 49 bits, K5 64); else 16 (KB2E_SAMPLER_TRIP16=1: tests)
            const int eb = std::max(1, bits_for(std::max<int64_t>(c->cfg.num_entities - 1, 1)));
            const int rb = std::max(1, bits_for(std::max<int64_t>(c->cfg.num_relations - 1, 1)));
            const bool pack = 2 * eb + rb + 10 <= 64 && !getenv("KB2E_SAMPLER_TRIP16");
            c->trip_eb = pack ? eb : 0;
            c->trip_rb = pack ? rb : 0;
            if (pack) {
                std::vector<uint64_t> tp((size_t)count);
                for (int64_t q = 0; q < count; ++q)
                    tp[q] = (uint64_t)h[q] | (uint64_t)t[q] << eb | (uint64_t)r[q] << (2 * eb) |
                            (uint64_t)thr[r[q]] << (2 * eb + rb);
                c->trip.alloc(tp.size() * 8);
                HIPCHK(hipMemcpy(c->trip.p, tp.data(), tp.size() * 8, hipMemcpyHostToDevice));
            } else {
                std::vector<int32_t> tp((size_t)count * 4);
                for (int64_t q = 0; q < count; ++q) {
                    tp[4 * q] = h[q];
                    tp[4 * q + 1] = t[q];
                    tp[4 * q + 2] = r[q];
                    tp[4 * q + 3] = thr[r[q]];
                }
                c->trip.alloc(tp.size() * 4);
                HIPCHK(hipMemcpy(c->trip.p, tp.data(), tp.size() * 4, hipMemcpyHostToDevice));
            }
        }
        if (c->cfg.model != KB2E_TRANSE && c->parallel()) {
            // PARALLEL TransH/TransR: every relation is its own event row
            c->plan.num_owners = c->cfg.num_relations;
            c->plan.owner.resize(c->cfg.num_relations);
            for (int r = 0; r < c->cfg.num_relations; ++r) c->plan.owner[r] = r;
        } else if (c->cfg.model != KB2E_TRANSE) {
            plan_owners(c->plan, c->ts, c->cfg.num_relations, c->num_cus);
        }
        setup_epoch_buffers(c);
        // setup used the legacy stream (hipMemset/hipMemcpy): the non-blocking
        // engine stream does not order against it, so drain it here
        HIPCHK(hipDeviceSynchronize());
        c->have_triples = true;
        c->epoch_pos = 0;
        c->epoch_ready = false;
        return KB2E_OK;
    });
}

kb2e_status kb2e_init_params(kb2e_ctx* c, double* ent_out, double* rel_out, double* w_out) {
    return guarded(c, [&] {
        HIPCHK(hipSetDevice(c->cfg.device));
        const int n = c->n;
        const int64_t ne = c->cfg.num_entities, nr = c->cfg.num_relations;
        std::vector<double> E((size_t)ne * n), R((size_t)nr * n), W((size_t)std::max<int64_t>(c->w_elems, 1));
        // initialEmbeddingValue: transe/trainer.cpp:21-23, transh/trainer.cpp:61-63, transr/trainer.cpp:66-68
        auto init = [&]() {
            if (c->cfg.model == KB2E_TRANSE)
                return randn(c->rng, 0, 1.0 / n, -6 / std::sqrt((double)n), 6 / std::sqrt((double)n));
            return randn(c->rng, 0, 1.0 / n, -1, 1);
        };
        auto norm_row = [&](double* a, bool ignore_short) {  // common/utils.cpp:70-77
            double res = 0;
            for (int i = 0; i < n; ++i) res += a[i] * a[i];
            double len = std::sqrt(res);
            if (!ignore_short || len > 1)
                for (int i = 0; i < n; ++i) a[i] /= len;
        };
        // common/trainer.cpp:45-57: relations first, then entities.
        for (int64_t i = 0; i < nr; ++i) {
            for (int j = 0; j < n; ++j) R[(size_t)i * n + j] = init();
            norm_row(&R[(size_t)i * n], true);
        }
        for (int64_t i = 0; i < ne; ++i) {
            for (int j = 0; j < n; ++j) E[(size_t)i * n + j] = init();
            norm_row(&E[(size_t)i * n], true);
        }
        if (c->cfg.model == KB2E_TRANSH) {  // transh/trainer.cpp:80-87
            for (int64_t i = 0; i < nr; ++i) {
                for (int j = 0; j < n; ++j) W[(size_t)i * n + j] = init();
                norm_row(&W[(size_t)i * n], false);
            }
        } else if (c->cfg.model == KB2E_TRANSR) {  // transr/trainer.cpp:73-86: identity
            for (int64_t i = 0; i < nr; ++i)
                for (int j = 0; j < n; ++j)
                    for (int k = 0; k < n; ++k) W[((size_t)i * n + j) * n + k] = (j == k) ? 1.0 : 0.0;
        }
        c->rng_version++;
        upload_tables(c, E.data(), R.data(), c->w_elems ? W.data() : nullptr);
        if (ent_out) std::memcpy(ent_out, E.data(), E.size() * 8);
        if (rel_out) std::memcpy(rel_out, R.data(), R.size() * 8);
        if (w_out && c->w_elems) std::memcpy(w_out, W.data(), (size_t)c->w_elems * 8);
        c->have_params = true;
        return KB2E_OK;
    });
}

kb2e_status kb2e_init_params_device(kb2e_ctx* c, double* ent_out, double* rel_out, double* w_out,
                                    int64_t* near_ties) {
    return guarded(c, [&] {
        HIPCHK(hipSetDevice(c->cfg.device));
        ensure_jump_table(c);
        const int n = c->n, model = c->cfg.model;
        const int64_t ne = c->cfg.num_entities, nr = c->cfg.num_relations;
        // common/trainer.cpp:45-57 relations then entities; transh/trainer.cpp:80-87 then the normals
        const int64_t rows = nr + ne + (model == KB2E_TRANSH ? nr : 0);
        DevBuf vals;
        vals.alloc((size_t)rows * n * 8);
        // initialEmbeddingValue: transe/trainer.cpp:21-23, transh/trainer.cpp:61-63, transr/trainer.cpp:66-68
        const double lim = model == KB2E_TRANSE ? 6 / std::sqrt((double)n) : 1.0;
        const int64_t ties = device_randn(c->rng, c->glibc_table.as<uint32_t>(), kGlibcBlock, 0, 1.0 / n, -lim, lim,
                                          rows * n, vals.as<double>(), c->stream);
        c->rng_version++;
        const double* v = vals.as<double>();
        place_rows(v, nr, n, c->ld, c->rel.p, c->f64(), true, true, c->stream);
        place_rows(v + nr * n, ne, n, c->ld, c->ent.p, c->f64(), true, true, c->stream);
        if (model == KB2E_TRANSH) place_rows(v + (nr + ne) * n, nr, n, c->ld, c->w.p, c->f64(), true, false, c->stream);
        if (model == KB2E_TRANSR) identity_weights(c->w.p, nr, n, c->ld, c->f64(), c->stream);
        HIPCHK(hipStreamSynchronize(c->stream));
        if (model == KB2E_TRANSR) sync_wsnap(c);
        c->have_params = true;
        if (near_ties) *near_ties = ties;
        if (ent_out || rel_out || w_out) return kb2e_download_params(c, ent_out, rel_out, w_out);
        return KB2E_OK;
    });
}

kb2e_status kb2e_transr_seed(kb2e_ctx* c, const double* e, const double* r) {
    return guarded(c, [&] {
        if (c->cfg.model != KB2E_TRANSR) return fail(c, KB2E_EUNSUPPORTED, "TransR only");
        if (!e || !r) return fail(c, KB2E_EINVAL, "entity and relation seed tables required");
        HIPCHK(hipSetDevice(c->cfg.device));
        const int n = c->n;
        std::vector<double> E(e, e + (size_t)c->cfg.num_entities * n);
        for (int64_t i = 0; i < c->cfg.num_entities; ++i) {  // common::norm(entityVec_[i], false)
            double* a = &E[(size_t)i * n];
            double res = 0;
            for (int j = 0; j < n; ++j) res += a[j] * a[j];
            const double len = std::sqrt(res);
            for (int j = 0; j < n; ++j) a[j] /= len;
        }
        upload_tables(c, E.data(), r, nullptr);
        return KB2E_OK;
    });
}

kb2e_status kb2e_upload_params(kb2e_ctx* c, const double* e, const double* r, const double* w) {
    return guarded(c, [&] {
        HIPCHK(hipSetDevice(c->cfg.device));
        if (!e || !r || (c->w_elems && !w && !c->have_params))
            return fail(c, KB2E_EINVAL, "entity, relation (and weight) tables required");
        upload_tables(c, e, r, w);
        c->have_params = true;
        return KB2E_OK;
    });
}

// ------------------------------------------------ text tables

namespace {
DevBuf* table_buf(kb2e_ctx* c, int32_t table, int64_t& rows) {
    rows = table == 0 ? c->cfg.num_entities : table == 1 ? c->cfg.num_relations : w_rows(c);
    if (table < 0 || table > 2 || rows == 0) throw std::invalid_argument("no such table for this model");
    return table == 0 ? &c->ent : table == 1 ? &c->rel : &c->w;
}
}  // namespace

kb2e_status kb2e_format_table(kb2e_ctx* c, int32_t table, char* buf, int64_t cap, int64_t* len) {
    return guarded(c, [&] {
        HIPCHK(hipSetDevice(c->cfg.device));
        HIPCHK(hipStreamSynchronize(c->stream));
        int64_t rows = 0;
        DevBuf* t = table_buf(c, table, rows);
        int64_t at = 0;
        const int64_t total = format_table(t->p, c->f64(), rows, c->n, c->ld, c->stream,
                                           [&](const char* p, size_t k) {
                                               if (buf && at + (int64_t)k <= cap) std::memcpy(buf + at, p, k);
                                               at += (int64_t)k;
                                           });
        if (len) *len = total;
        if (!buf || total > cap) return fail(c, KB2E_EINVAL, "buffer too small for the formatted table");
        return KB2E_OK;
    });
}

kb2e_status kb2e_write_table(kb2e_ctx* c, int32_t table, const char* path) {
    return guarded(c, [&] {
        HIPCHK(hipSetDevice(c->cfg.device));
        HIPCHK(hipStreamSynchronize(c->stream));
        int64_t rows = 0;
        DevBuf* t = table_buf(c, table, rows);
        FILE* f = path ? std::fopen(path, "w") : nullptr;
        if (!f) return fail(c, KB2E_EINVAL, std::string("could not open output file: ") + (path ? path : "(null)"));
        bool ok = true;
        format_table(t->p, c->f64(), rows, c->n, c->ld, c->stream,
                     [&](const char* p, size_t k) { ok = ok && std::fwrite(p, 1, k, f) == k; });
        ok = (std::fclose(f) == 0) && ok;
        if (!ok) return fail(c, KB2E_EINVAL, std::string("write failed: ") + path);
        return KB2E_OK;
    });
}

kb2e_status kb2e_read_table(kb2e_ctx* c, int32_t table, const char* path, int32_t mode) {
    return guarded(c, [&] {
        HIPCHK(hipSetDevice(c->cfg.device));
        if (mode < KB2E_READ_VERBATIM || mode > KB2E_READ_SHRINK) return fail(c, KB2E_EINVAL, "bad read mode");
        int64_t rows = 0;
        DevBuf* t = table_buf(c, table, rows);
        FILE* f = path ? std::fopen(path, "rb") : nullptr;
        if (!f) return fail(c, KB2E_EINVAL, std::string("could not open table file: ") + (path ? path : "(null)"));
        std::vector<char> text;
        char chunk[1 << 16];
        size_t k;
        while ((k = std::fread(chunk, 1, sizeof chunk, f)) > 0) text.insert(text.end(), chunk, chunk + k);
        std::fclose(f);
        const int64_t count = rows * c->n;
        DevBuf vals;
        vals.alloc((size_t)count * 8);
        HIPCHK(hipStreamSynchronize(c->stream));
        int64_t bad = -1, slow = 0;
        const int64_t got = parse_doubles(text.data(), (int64_t)text.size(), count, vals.as<double>(), c->stream,
                                          &bad, &slow);
        if (got < count)
            return fail(c, KB2E_EINVAL, std::string("Failed to read embedding values from seed file: '") + path + "'");
        place_rows(vals.as<double>(), rows, c->n, c->ld, t->p, c->f64(), mode != KB2E_READ_VERBATIM,
                   mode == KB2E_READ_SHRINK, c->stream);
        HIPCHK(hipStreamSynchronize(c->stream));
        if (table == 2) sync_wsnap(c);
        // tables loaded from text alone (the evaluators) are complete once every table the model has is read
        c->tables_read |= 1 << table;
        if ((c->tables_read & 3) == 3 && (!c->w_elems || (c->tables_read & 4))) c->have_params = true;
        return KB2E_OK;
    });
}

kb2e_status kb2e_download_params(kb2e_ctx* c, double* e, double* r, double* w) {
    return guarded(c, [&] {
        HIPCHK(hipSetDevice(c->cfg.device));
        HIPCHK(hipStreamSynchronize(c->stream));
        check_dataflow(c);  // tables a timed-out wait left are not handed out
        const int64_t ne = c->cfg.num_entities, nr = c->cfg.num_relations;
        if (c->f64()) {
            if (e) download_rows<double>(c, c->ent, e, ne, c->n, c->ld);
            if (r) download_rows<double>(c, c->rel, r, nr, c->n, c->ld);
            if (w && w_rows(c)) download_rows<double>(c, c->w, w, w_rows(c), c->n, c->ld);
        } else {
            if (e) download_rows<float>(c, c->ent, e, ne, c->n, c->ld);
            if (r) download_rows<float>(c, c->rel, r, nr, c->n, c->ld);
            if (w && w_rows(c)) download_rows<float>(c, c->w, w, w_rows(c), c->n, c->ld);
        }
        return KB2E_OK;
    });
}

kb2e_status kb2e_get_transr_work(kb2e_ctx* c, double* hw, double* tw) {
    return guarded(c, [&] {
        if (c->cfg.model != KB2E_TRANSR) return fail(c, KB2E_EUNSUPPORTED, "TransR only");
        HIPCHK(hipStreamSynchronize(c->stream));
        std::vector<double> h(2 * (size_t)c->n);
        HIPCHK(hipMemcpy(h.data(), c->transr_work.p, h.size() * 8, hipMemcpyDeviceToHost));
        std::memcpy(hw, h.data(), (size_t)c->n * 8);
        std::memcpy(tw, h.data() + c->n, (size_t)c->n * 8);
        return KB2E_OK;
    });
}

kb2e_status kb2e_set_transr_work(kb2e_ctx* c, const double* hw, const double* tw) {
    return guarded(c, [&] {
        if (c->cfg.model != KB2E_TRANSR) return fail(c, KB2E_EUNSUPPORTED, "TransR only");
        if (!c->have_triples) return fail(c, KB2E_ESTATE, "upload triples first");
        std::vector<double> h(2 * (size_t)c->n);
        std::memcpy(h.data(), hw, (size_t)c->n * 8);
        std::memcpy(h.data() + c->n, tw, (size_t)c->n * 8);
        HIPCHK(hipStreamSynchronize(c->stream));
        HIPCHK(hipMemcpy(c->transr_work.p, h.data(), h.size() * 8, hipMemcpyHostToDevice));
        return KB2E_OK;
    });
}

kb2e_status kb2e_set_sample_stream(kb2e_ctx* c, const int32_t* i, const int32_t* j, const uint8_t* side,
                                   int64_t count) {
    return guarded(c, [&] {
        if (!c->have_triples) return fail(c, KB2E_ESTATE, "upload triples first");
        for (int64_t k = 0; k < count; ++k)
            if (i[k] < 0 || i[k] >= c->ts.size() || j[k] < 0 || j[k] >= c->cfg.num_entities)
                return fail(c, KB2E_EINVAL, "sample " + std::to_string(k) + " out of range");
        c->rp_si.assign(i, i + count);
        c->rp_sj.assign(j, j + count);
        c->rp_side.assign(side, side + count);
        c->rp_pos = 0;
        return KB2E_OK;
    });
}

kb2e_status kb2e_get_sample_stream(kb2e_ctx* c, int32_t* i, int32_t* j, uint8_t* side, int64_t count) {
    return guarded(c, [&] {
        if (!c->epoch_ready) return fail(c, KB2E_ESTATE, "no epoch in progress");
        const int64_t k = std::min<int64_t>(count, c->S);
        HIPCHK(hipStreamSynchronize(c->stream));
        HIPCHK(hipMemcpy(i, c->si(), k * 4, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(j, c->sj(), k * 4, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(side, c->side(), k, hipMemcpyDeviceToHost));
        return KB2E_OK;
    });
}

kb2e_status kb2e_train_batches(kb2e_ctx* c, int32_t nbatches) {
    return guarded(c, [&] {
        if (!c->have_triples || !c->have_params) return fail(c, KB2E_ESTATE, "upload triples and params first");
        HIPCHK(hipSetDevice(c->cfg.device));
        run_batches(c, nbatches);
        return KB2E_OK;
    });
}

kb2e_status kb2e_synchronize(kb2e_ctx* c) {
    return guarded(c, [&] {
        HIPCHK(hipStreamSynchronize(c->stream));
        // the next epoch's sampling / index, queued on the side stream during
        // this one, is part of the work the caller waits for
        if (c->side_stream) HIPCHK(hipStreamSynchronize(c->side_stream));
        check_dataflow(c);  // a bounded in-kernel wait that timed out fails here, not only in take_stats
        return KB2E_OK;
    });
}

kb2e_status kb2e_take_stats(kb2e_ctx* c, double* loss, int64_t* active) {
    return guarded(c, [&] {
        if (c->have_triples) {
            reduce_stats(c, c->epoch_pos * c->B);
            collect_stats(c);
        }
#ifdef KB2E_OWNER_PROF
        {
            std::vector<unsigned long long> pr((size_t)kProfOwners * 16);
            HIPCHK(hipMemcpyFromSymbol(pr.data(), HIP_SYMBOL(g_owner_prof), pr.size() * 8));
            for (int o = 0; o < kProfOwners; ++o) {
                if (!pr[(size_t)o * 16 + 11]) continue;
                fprintf(stderr, "owner_prof %d", o);
                for (int k = 0; k < 16; ++k) fprintf(stderr, " %llu", pr[(size_t)o * 16 + k]);
                fprintf(stderr, "\n");
            }
            std::fill(pr.begin(), pr.end(), 0ull);
            HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_owner_prof), pr.data(), pr.size() * 8));
            unsigned long long fp[2][16];
            HIPCHK(hipMemcpyFromSymbol(fp, HIP_SYMBOL(g_fold_prof), sizeof(fp)));
            for (int g = 0; g < 2; ++g) {
                fprintf(stderr, "fold_prof %d", g);
                for (int k = 0; k < 16; ++k) fprintf(stderr, " %llu", fp[g][k]);
                fprintf(stderr, "\n");
            }
            std::memset(fp, 0, sizeof(fp));
            HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_fold_prof), fp, sizeof(fp)));
            HIPCHK(hipMemcpyFromSymbol(fp[0], HIP_SYMBOL(g_long_prof), sizeof(fp[0])));
            fprintf(stderr, "long_prof");
            for (int k = 0; k < 16; ++k) fprintf(stderr, " %llu", fp[0][k]);
            fprintf(stderr, "\n");
            HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_long_prof), fp[1], sizeof(fp[1])));
        }
#endif
        if (getenv("KB2E_RPAR_STATS")) {  // transRNorm rounds of the PARALLEL TransR schedule
            unsigned long long st[16];
            HIPCHK(hipMemcpyFromSymbol(st, HIP_SYMBOL(g_rpar_rounds), sizeof(st)));
            cons_wave_take_stats(st);  // the register-resident kernel's own counters
            fprintf(stderr, "rpar_rounds rounds of row blocks %llu, tiles with violators %llu, most rounds of a block %llu\n",
                    st[0], st[1], st[2]);
            fprintf(stderr, "rpar_cons cycles: setup %llu, P0+rounds %llu, records %llu, longest block %llu, blocks %llu\n",
                    st[3], st[4], st[5], st[6], st[7]);
            if (c->rpar_cons_seq || c->rpar_cons_wide) {
                unsigned long long q[64];
                cons_seq_take_stats(q);
                fprintf(stderr, "rpar_cons chunk kernel: relations %llu, chunks %llu (most in a relation %llu), "
                        "violators %llu, rounds %llu (most %llu), cycles mean %.0f max %llu\n", q[0], q[1], q[6], q[2],
                        q[3], q[7], q[0] ? (double)q[4] / (double)q[0] : 0.0, q[5]);
                if (c->rpar_cons_wide && cons_chainw_pipelined(c->n))
                    fprintf(stderr, "rpar_cons pipelined wide chain phases (walker: prologue+K0, window list, walk, "
                            "B1 wait, row stores+fold, B2 wait, drain, window flags, tail, write-back+records, -; helper: "
                            "debt+fold+B2, X tile, B1 wait; walker: row+V, sums+rounds+g, later rows):");
                else if (c->rpar_cons_wide)
                    fprintf(stderr, "rpar_cons wide chain phases (prologue, window list, rows+barrier, P+Gram+B1, "
                            "K0, V+sums, B(1), rounds+g, B(2), later pairs, B(3), records+W update, chunk barrier, "
                            "window flags, tail, write-back):");
                else  // (the tick indices of kernels_transr_pipe.hpp; the serial kernel's differ, kernels_transr_seq.hpp)
                    fprintf(stderr, "rpar_cons chunk phases (prologue, chunk start, walk end + publish, B1 wait, "
                            "pick + row to LDS, helper B1 wait, after B1, V, sums, rounds + g, g store, later rows; helper wave 1: debt, tiles, "
                            "helper_sync wait, rows + corrections):");
                for (int k = 8; k < 24; ++k) fprintf(stderr, " %llu", q[k]);
                fprintf(stderr, "; hot relations (%llu, %llu chunks, %llu violators):", q[41], q[40], q[42]);
                for (int k = 24; k < 40; ++k) fprintf(stderr, " %llu", q[k]);
                fprintf(stderr, "\n");
            }
            if (c->rpar_cons_wave)
                fprintf(stderr, "rpar_cons wave kernel: longest setup %llu, P0+rounds %llu, records %llu, a wave's "
                        "rounds %llu; MFMA rounds before the VALU tail %llu, blocks entering it %llu\n",
                        st[8], st[9], st[10], st[11], st[12], st[13]);
            else
                fprintf(stderr, "rpar_rounds wave 0: loads+mfma issue %llu, barriers %llu, update part %llu, lockstep "
                        "rounds %llu, tail %llu, G+ballot %llu\n", st[8], st[9], st[10], st[11], st[12], st[13]);
            std::memset(st, 0, sizeof(st));
            HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_rpar_rounds), st, sizeof(st)));
        }
        if (loss) *loss = c->acc_loss;
        if (active) *active = c->acc_active;
        c->acc_loss = 0;
        c->acc_active = 0;
        return KB2E_OK;
    });
}

kb2e_status kb2e_train_epoch(kb2e_ctx* c, double* loss, int64_t* active) {
    return guarded(c, [&] {
        if (!c->have_triples || !c->have_params) return fail(c, KB2E_ESTATE, "upload triples and params first");
        if (c->epoch_pos != 0) return fail(c, KB2E_ESTATE, "an epoch is partially trained (kb2e_train_batches)");
        HIPCHK(hipSetDevice(c->cfg.device));
        c->acc_loss = 0;
        c->acc_active = 0;
        HIPCHK(hipMemsetAsync(c->stats.p, 0, 16, c->stream));  // only this epoch's statistics
        run_batches(c, c->nb);
        collect_stats(c);
        if (loss) *loss = c->acc_loss;
        if (active) *active = c->acc_active;
        c->acc_loss = 0;
        c->acc_active = 0;
        return KB2E_OK;
    });
}

namespace {
EvalTables eval_tables(kb2e_ctx* c) {
    EvalTables t{};
    t.model = c->cfg.model;
    t.n = c->n;
    t.ld = c->ld;
    t.ne = c->cfg.num_entities;
    t.nr = c->cfg.num_relations;
    t.l1 = c->cfg.distance == 0 || c->cfg.model == KB2E_TRANSH;
    t.f64 = c->f64();
    t.ent = c->ent.p;
    t.rel = c->rel.p;
    // ORDERED TransR keeps the committed matrices in wsnap (W_A)
    t.w = c->cfg.model == KB2E_TRANSR && !c->parallel() ? c->wsnap.p : c->w.p;
    t.stream = c->stream;
    return t;
}
}  // namespace

kb2e_status kb2e_evaluate(kb2e_ctx* c, const int32_t* th, const int32_t* tt, const int32_t* tr, int64_t ntest,
                          const int32_t* fh, const int32_t* ft, const int32_t* fr, int64_t nfilter, double* out) {
    return guarded(c, [&] {
        if (!th || !tt || !tr || ntest < 1 || !out || (nfilter > 0 && (!fh || !ft || !fr)))
            return fail(c, KB2E_EINVAL, "empty test set");
        if (!c->have_params) return fail(c, KB2E_ESTATE, "no embeddings on the device");
        HIPCHK(hipSetDevice(c->cfg.device));
        c->timed("eval", [&] { evaluate_fixed(eval_tables(c), EvalQuery{th, tt, tr, ntest, fh, ft, fr, nfilter}, out); });
        return KB2E_OK;
    });
}

kb2e_status kb2e_evaluate_transr_compat(kb2e_ctx* c, const int32_t* th, const int32_t* tt, const int32_t* tr,
                                        int64_t ntest, const int32_t* fh, const int32_t* ft, const int32_t* fr,
                                        int64_t nfilter, double* work, double* out,
                                        void (*progress)(double fraction, void* user), void* user) {
    return guarded(c, [&] {
        if (!th || !tt || !tr || ntest < 1 || !out || (nfilter > 0 && (!fh || !ft || !fr)))
            return fail(c, KB2E_EINVAL, "empty test set");
        if (c->cfg.model != KB2E_TRANSR) return fail(c, KB2E_EUNSUPPORTED, "TransR only");
        if (!c->have_params) return fail(c, KB2E_ESTATE, "no embeddings on the device");
        HIPCHK(hipSetDevice(c->cfg.device));
        c->timed("eval", [&] {
            evaluate_transr_compat(eval_tables(c), EvalQuery{th, tt, tr, ntest, fh, ft, fr, nfilter}, work, out,
                                   progress, user);
        });
        return KB2E_OK;
    });
}

int32_t kb2e_rng_next(kb2e_ctx* c) {
    if (!c) return -1;
    c->rng_version++;
    return c->rng.next();
}

kb2e_status kb2e_profile_enable(kb2e_ctx* c, int32_t on) {
    return guarded(c, [&] {
        c->flush_timers();
        c->prof = on != 0;
        c->prof_period = on > 1 ? on : 1;
        c->prof_counter = 0;
        c->timers.clear();
        return KB2E_OK;
    });
}

kb2e_status kb2e_profile_query(kb2e_ctx* c, const char* name, double* total_ms, int64_t* launches) {
    return guarded(c, [&] {
        c->flush_timers();
        auto it = c->timers.find(name ? name : "");
        if (total_ms) *total_ms = it == c->timers.end() ? 0.0 : it->second.ms;
        if (launches) *launches = it == c->timers.end() ? 0 : it->second.launches;
        return KB2E_OK;
    });
}

kb2e_status kb2e_counter(kb2e_ctx* c, const char* name, int64_t* value) {
    return guarded(c, [&] {
        const std::string nm = name ? name : "";
        if (nm != "transh_orth_rel_batches" || !value) return fail(c, KB2E_EINVAL, "unknown counter '" + nm + "'");
        *value = 0;
        if (!c->hpar_count.p) return KB2E_OK;  // (not a PARALLEL TransH context, or no triples yet)
        uint32_t v = 0;
        HIPCHK(hipStreamSynchronize(c->stream));
        HIPCHK(hipMemcpy(&v, (const uint32_t*)c->hpar_count.p + 2, 4, hipMemcpyDeviceToHost));
        *value = v;
        return KB2E_OK;
    });
}

int64_t kb2e_device_bytes(const kb2e_ctx* c) { return c ? c->device_bytes : 0; }

kb2e_status kb2e_device_tables(kb2e_ctx* c, void** e, void** r, void** w, int64_t* ne, int64_t* nr, int64_t* nw) {
    return guarded(c, [&] {
        if (e) *e = c->ent.p;
        if (r) *r = c->rel.p;
        if (w) *w = c->w_elems ? c->w.p : nullptr;
        if (ne) *ne = (int64_t)c->cfg.num_entities * c->ld;
        if (nr) *nr = (int64_t)c->cfg.num_relations * c->ld;
        if (nw) *nw = c->w_elems ? w_rows(c) * c->ld : 0;
        return KB2E_OK;
    });
}

kb2e_status kb2e_renormalize(kb2e_ctx* c, const uint8_t* ent_rows, const uint8_t* rel_rows, const uint8_t* w_rows) {
    return guarded(c, [&] {
        HIPCHK(hipSetDevice(c->cfg.device));
        const uint8_t* masks[3] = {ent_rows, rel_rows, w_rows};
        const int ntab = c->cfg.model == KB2E_TRANSE ? 2 : 3;
        DevBuf mbuf;
        for (int t = 0; t < ntab; ++t) {
            const int64_t units = t == 0 ? c->cfg.num_entities : c->cfg.num_relations;
            const uint8_t* dmask = nullptr;
            if (masks[t]) {
                mbuf.alloc(units);
                HIPCHK(hipMemcpyAsync(mbuf.p, masks[t], units, hipMemcpyHostToDevice, c->stream));
                dmask = mbuf.as<uint8_t>();
            }
            renorm_rows(c, t, 0, units, dmask);
            HIPCHK(hipStreamSynchronize(c->stream));  // mbuf is reused
        }
        sync_wsnap(c);
        return KB2E_OK;
    });
}

kb2e_status kb2e_renormalize_rows(kb2e_ctx* c, int32_t table, int64_t first, int64_t count,
                                  const uint8_t* device_mask) {
    return guarded(c, [&] {
        const int ntab = c->cfg.model == KB2E_TRANSE ? 2 : 3;
        if (table < 0 || table >= ntab) return fail(c, KB2E_EINVAL, "no such table");
        const int64_t units = table == 0 ? c->cfg.num_entities : c->cfg.num_relations;
        if (first < 0 || count < 0 || first + count > units) return fail(c, KB2E_EINVAL, "rows out of range");
        HIPCHK(hipSetDevice(c->cfg.device));
        renorm_rows(c, table, first, count, device_mask);
        HIPCHK(hipStreamSynchronize(c->stream));
        if (table == 2) sync_wsnap(c);  // TransR: the committed matrices follow
        return KB2E_OK;
    });
}

}  // extern "C"

#include "engine_merge.inc"
