/*
 * oracle/orc.c -- CPU restatement of eriq-augustine/KB2E training/evaluation.
 * TEST INFRASTRUCTURE ONLY (see orc.h).  Compiled with -ffp-contract=off so
 * every multiply/add rounds exactly as the reference's x86-64 SSE2 build does.
 */
#define _DEFAULT_SOURCE
#include "orc.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define ORC_PI 3.1415926535897932384626433832795 /* common/utils.h:8 */

struct orc_model {
    int model, n, ne, nr;
    double lr, margin;
    int method, distance, nbatches, transr_compat;
    /* Trainer::heads_/tails_/relations_ (common/trainer.h:43-45) */
    int ntrain;
    int *heads, *tails, *rels;
    /* Trainer::triples_ (common/trainer.h:49): sorted (h, r, t) keys */
    uint64_t* filter;
    long long nfilter;
    /* relation{Head,Tail}MeanCooccurrence_ (common/trainer.h:53-55) */
    double *head_mean, *tail_mean;
    /* snapshot + next tables (transe/trainer.h:17-18, transh/trainer.h:14-19,
     * transr/trainer.h:31-36) */
    double *ent, *rel, *w;
    double *ent_next, *rel_next, *w_next;
    long long wsize; /* elements of w */
    /* transr::Trainer::headWorkVec_/tailWorkVec_ (transr/trainer.h:28-29) */
    double *hwork, *twork;
};

/* The reference's RNG is glibc rand() (TYPE_3 random_r on a global state).
 * The oracle keeps a PRIVATE TYPE_3 state and draws with random_r: the same
 * algorithm and stream, but immune to other rand() callers in the process
 * (the HIP runtime draws from the global state while it initialises). */
static struct random_data g_rd;
static char g_rstate[128];  /* 128 bytes selects TYPE_3, glibc's rand() default */
static int g_rinit = 0;

static long long g_orth_iters = 0;
static long long g_site_iters[4];
static int g_site = 3;
static long long g_transr_norm_iters = 0;

/* ------------------------------------------------------------------ L0 */

void orc_srand(unsigned seed) {
    if (!g_rinit) {
        memset(&g_rd, 0, sizeof(g_rd));
        initstate_r(seed, g_rstate, sizeof(g_rstate), &g_rd);
        g_rinit = 1;
    }
    srandom_r(seed, &g_rd);
}

int orc_rand(void) {
    int32_t r;
    if (!g_rinit) orc_srand(1); /* glibc: rand() without srand() behaves as srand(1) */
    random_r(&g_rd, &r);
    return (int)r;
}

/* common/utils.cpp:18-20 */
double orc_rand_range(double min, double max) {
    return min + (max - min) * orc_rand() / (RAND_MAX + 1.0);
}

static double sqr(double x) { return x * x; } /* common/utils.cpp:40-42 */

/* common/utils.cpp:22-24 */
double orc_normal(double x, double miu, double sigma) {
    return 1.0 / sqrt(2 * ORC_PI) / sigma * exp(-1 * sqr(x - miu) / (2 * sqr(sigma)));
}

/* common/utils.cpp:26-38 */
double orc_randn(double miu, double sigma, double min, double max) {
    double x, y, dScope;
    do {
        x = orc_rand_range(min, max);
        y = orc_normal(x, miu, sigma);
        dScope = orc_rand_range(0.0, orc_normal(miu, miu, sigma));
    } while (dScope > y);
    return x;
}

/* common/utils.cpp:113-120: (rand()*rand()) % x in int32 with wrap-around. */
int orc_randmax(int x) {
    unsigned a = (unsigned)orc_rand();
    unsigned b = (unsigned)orc_rand();
    int res = (int)(a * b) % x;
    while (res < 0) res += x;
    return res;
}

/* common/utils.cpp:44-51 */
double orc_vec_len(const double* a, int n) {
    double res = 0;
    for (int i = 0; i < n; i++) res += sqr(a[i]);
    return sqrt(res);
}

/* common/utils.cpp:70-77 */
void orc_norm(double* a, int n, int ignore_short) {
    double len = orc_vec_len(a, n);
    if (!ignore_short || len > 1) {
        for (int i = 0; i < n; i++) a[i] /= len;
    }
}

/* common/utils.cpp:79-111 (note: `sum` is never reset between iterations) */
void orc_norm_orth(double* a, double* b, int n, double rate) {
    orc_norm(b, n, 0);
    double sum = 0;
    while (1) {
        for (int i = 0; i < n; i++) sum += sqr(b[i]);
        sum = sqrt(sum);
        for (int i = 0; i < n; i++) b[i] /= sum;
        double x = 0;
        for (int i = 0; i < n; i++) x += b[i] * a[i];
        if (x > 0.1) {
            g_orth_iters++;
            g_site_iters[g_site]++;
            for (int i = 0; i < n; i++) {
                a[i] -= rate * b[i];
                b[i] -= rate * a[i];
            }
        } else {
            break;
        }
    }
    orc_norm(b, n, 0);
}

long long orc_norm_orth_iterations(void) { return g_orth_iters; }
/* instrumentation: coupling-loop iterations per call site (0 = relation / head,
 * 1 = head / tail, 2 = tail / entity[relation], 3 = direct calls) */
long long orc_site_iterations(int site) { return (site >= 0 && site < 4) ? g_site_iters[site] : 0; }

/* transr/trainer.cpp:35-64; b is n x n with b[j*n+i] = weights[j][i]. */
void orc_transr_norm(double* a, double* b, int n, double rate) {
    while (1) {
        double x = 0;
        for (int i = 0; i < n; i++) {
            double tmp = 0;
            for (int j = 0; j < n; j++) tmp += b[j * n + i] * a[j];
            x += sqr(tmp);
        }
        if (x <= 1) break;
        g_transr_norm_iters++;
        g_site_iters[g_site]++;
        double lambda = 1;
        for (int i = 0; i < n; i++) {
            double tmp = 0;
            for (int j = 0; j < n; j++) tmp += b[j * n + i] * a[j];
            tmp *= 2;
            for (int j = 0; j < n; j++) {
                b[j * n + i] -= rate * lambda * tmp * a[j];
                a[j] -= rate * lambda * tmp * b[j * n + i];
            }
        }
    }
}

long long orc_transr_norm_iterations(void) { return g_transr_norm_iters; }

/* ------------------------------------------------------------ lifecycle */

static void* xcalloc(size_t n, size_t s) {
    void* p = calloc(n ? n : 1, s);
    if (!p) {
        fprintf(stderr, "orc: out of memory\n");
        abort();
    }
    return p;
}

orc_model* orc_create(int model, int dim, int num_entities, int num_relations,
                      double learning_rate, double margin, int method, int distance,
                      int num_batches, int transr_compat) {
    orc_model* m = (orc_model*)xcalloc(1, sizeof(orc_model));
    m->model = model;
    m->n = dim;
    m->ne = num_entities;
    m->nr = num_relations;
    m->lr = learning_rate;
    m->margin = margin;
    m->method = method;
    m->distance = distance;
    m->nbatches = num_batches;
    m->transr_compat = transr_compat;
    size_t n = (size_t)dim;
    m->ent = (double*)xcalloc((size_t)num_entities * n, sizeof(double));
    m->rel = (double*)xcalloc((size_t)num_relations * n, sizeof(double));
    m->ent_next = (double*)xcalloc((size_t)num_entities * n, sizeof(double));
    m->rel_next = (double*)xcalloc((size_t)num_relations * n, sizeof(double));
    if (model == ORC_TRANSH) m->wsize = (long long)num_relations * dim;
    if (model == ORC_TRANSR) m->wsize = (long long)num_relations * dim * dim;
    m->w = (double*)xcalloc((size_t)m->wsize, sizeof(double));
    m->w_next = (double*)xcalloc((size_t)m->wsize, sizeof(double));
    m->hwork = (double*)xcalloc(n, sizeof(double));
    m->twork = (double*)xcalloc(n, sizeof(double));
    return m;
}

void orc_destroy(orc_model* m) {
    if (!m) return;
    free(m->heads); free(m->tails); free(m->rels); free(m->filter);
    free(m->head_mean); free(m->tail_mean);
    free(m->ent); free(m->rel); free(m->w);
    free(m->ent_next); free(m->rel_next); free(m->w_next);
    free(m->hwork); free(m->twork);
    free(m);
}

static uint64_t fkey(const orc_model* m, int h, int r, int t) {
    return ((uint64_t)h * (uint64_t)m->nr + (uint64_t)r) * (uint64_t)m->ne + (uint64_t)t;
}

static int cmp_u64(const void* a, const void* b) {
    uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
    return x < y ? -1 : (x > y ? 1 : 0);
}

static int cmp_int(const void* a, const void* b) {
    int x = *(const int*)a, y = *(const int*)b;
    return x < y ? -1 : (x > y ? 1 : 0);
}

static int filter_has(const uint64_t* keys, long long n, uint64_t k) {
    long long lo = 0, hi = n;
    while (lo < hi) {
        long long mid = (lo + hi) >> 1;
        if (keys[mid] < k) lo = mid + 1; else hi = mid;
    }
    return lo < n && keys[lo] == k;
}

int orc_in_train(const orc_model* m, int h, int r, int t) {
    return filter_has(m->filter, m->nfilter, fkey(m, h, r, t));
}

/* Trainer::add (common/trainer.cpp:26-32) for every triple, then the
 * co-occurrence means of Trainer::loadFiles (common/trainer.cpp:163-194). */
int orc_set_triples(orc_model* m, const int* heads, const int* tails, const int* rels, int count) {
    m->ntrain = count;
    m->heads = (int*)xcalloc((size_t)count, sizeof(int));
    m->tails = (int*)xcalloc((size_t)count, sizeof(int));
    m->rels = (int*)xcalloc((size_t)count, sizeof(int));
    memcpy(m->heads, heads, sizeof(int) * (size_t)count);
    memcpy(m->tails, tails, sizeof(int) * (size_t)count);
    memcpy(m->rels, rels, sizeof(int) * (size_t)count);

    m->filter = (uint64_t*)xcalloc((size_t)count, sizeof(uint64_t));
    for (int k = 0; k < count; k++) m->filter[k] = fkey(m, heads[k], rels[k], tails[k]);
    qsort(m->filter, (size_t)count, sizeof(uint64_t), cmp_u64);
    long long u = 0;
    for (long long k = 0; k < count; k++)
        if (k == 0 || m->filter[k] != m->filter[k - 1]) m->filter[u++] = m->filter[k];
    m->nfilter = u;

    /* headCooccurrence[relation][head]++ / tailCooccurrence[relation][tail]++
     * (common/trainer.cpp:163-167); mean = total / distinct (:171-194). */
    m->head_mean = (double*)xcalloc((size_t)m->nr, sizeof(double));
    m->tail_mean = (double*)xcalloc((size_t)m->nr, sizeof(double));
    int* order = (int*)xcalloc((size_t)count, sizeof(int));
    for (int side = 0; side < 2; side++) {
        /* sort (relation, entity) pairs to count distinct entities per relation */
        uint64_t* pairs = (uint64_t*)xcalloc((size_t)count, sizeof(uint64_t));
        for (int k = 0; k < count; k++)
            pairs[k] = ((uint64_t)rels[k] << 32) | (uint32_t)(side == 0 ? heads[k] : tails[k]);
        qsort(pairs, (size_t)count, sizeof(uint64_t), cmp_u64);
        double* out = side == 0 ? m->head_mean : m->tail_mean;
        long long k = 0;
        while (k < count) {
            int r = (int)(pairs[k] >> 32);
            double total = 0;
            long long distinct = 0;
            while (k < count && (int)(pairs[k] >> 32) == r) {
                long long e = k;
                while (e < count && pairs[e] == pairs[k]) e++;
                distinct++;
                total += (double)(e - k);
                k = e;
            }
            /* the reference sums per-entity counts in entity order; all counts are
             * small integers so the double sum is exact in any order */
            if (r >= 0 && r < m->nr) out[r] = total / (double)distinct;
        }
        free(pairs);
    }
    free(order);
    (void)cmp_int;
    return 0;
}

int orc_batch_size(const orc_model* m) { return m->ntrain / m->nbatches; }

static double initial_value(const orc_model* m) {
    if (m->model == ORC_TRANSE) /* transe/trainer.cpp:21-23 */
        return orc_randn(0, 1.0 / m->n, -6 / sqrt((double)m->n), 6 / sqrt((double)m->n));
    /* transh/trainer.cpp:61-63, transr/trainer.cpp:66-68 */
    return orc_randn(0, 1.0 / m->n, -1, 1);
}

/* common/trainer.cpp:34-58 (+ transh/trainer.cpp:77-88, transr/trainer.cpp:70-86) */
void orc_prep_train(orc_model* m) {
    int n = m->n;
    for (int i = 0; i < m->nr; i++) {
        for (int j = 0; j < n; j++) m->rel[(size_t)i * n + j] = initial_value(m);
        orc_norm(m->rel + (size_t)i * n, n, 1);
    }
    for (int i = 0; i < m->ne; i++) {
        for (int j = 0; j < n; j++) m->ent[(size_t)i * n + j] = initial_value(m);
        orc_norm(m->ent + (size_t)i * n, n, 1);
    }
    if (m->model == ORC_TRANSH) {
        for (int i = 0; i < m->nr; i++) {
            for (int j = 0; j < n; j++) m->w[(size_t)i * n + j] = initial_value(m);
            orc_norm(m->w + (size_t)i * n, n, 0);
        }
    } else if (m->model == ORC_TRANSR) {
        for (int i = 0; i < m->nr; i++)
            for (int j = 0; j < n; j++)
                for (int k = 0; k < n; k++)
                    m->w[((size_t)i * n + j) * n + k] = (k == j) ? 1.0 : 0.0;
    }
}

/* transr/trainer.cpp:88-113 */
void orc_transr_seed(orc_model* m, const double* ent, const double* rel) {
    size_t n = (size_t)m->n;
    memcpy(m->ent, ent, sizeof(double) * (size_t)m->ne * n);
    for (int i = 0; i < m->ne; i++) orc_norm(m->ent + (size_t)i * n, m->n, 0);
    memcpy(m->rel, rel, sizeof(double) * (size_t)m->nr * n);
}

void orc_get_tables(const orc_model* m, double* ent, double* rel, double* w) {
    size_t n = (size_t)m->n;
    if (ent) memcpy(ent, m->ent, sizeof(double) * (size_t)m->ne * n);
    if (rel) memcpy(rel, m->rel, sizeof(double) * (size_t)m->nr * n);
    if (w && m->wsize) memcpy(w, m->w, sizeof(double) * (size_t)m->wsize);
}

void orc_set_tables(orc_model* m, const double* ent, const double* rel, const double* w) {
    size_t n = (size_t)m->n;
    if (ent) memcpy(m->ent, ent, sizeof(double) * (size_t)m->ne * n);
    if (rel) memcpy(m->rel, rel, sizeof(double) * (size_t)m->nr * n);
    if (w && m->wsize) memcpy(m->w, w, sizeof(double) * (size_t)m->wsize);
}

void orc_get_transr_work(const orc_model* m, double* hwork, double* twork) {
    memcpy(hwork, m->hwork, sizeof(double) * (size_t)m->n);
    memcpy(twork, m->twork, sizeof(double) * (size_t)m->n);
}

void orc_set_transr_work(orc_model* m, const double* hwork, const double* twork) {
    memcpy(m->hwork, hwork, sizeof(double) * (size_t)m->n);
    memcpy(m->twork, twork, sizeof(double) * (size_t)m->n);
}

/* ------------------------------------------------------------ energies */

#define ROW(t, i) ((t) + (size_t)(i) * (size_t)m->n)

/* transe/transe.cpp:10-28 */
static double transe_energy(const orc_model* m, const double* E, const double* R, int h, int t, int r) {
    const double *eh = ROW(E, h), *et = ROW(E, t), *er = ROW(R, r);
    double energy = 0;
    if (m->distance == 0) {
        for (int i = 0; i < m->n; i++) energy += fabs(et[i] - eh[i] - er[i]);
    } else {
        for (int i = 0; i < m->n; i++) energy += sqr(et[i] - eh[i] - er[i]);
    }
    return energy;
}

/* transh/transh.cpp:10-29 (always L1) */
static double transh_energy(const orc_model* m, const double* E, const double* R, const double* W,
                            int h, int t, int r) {
    const double *eh = ROW(E, h), *et = ROW(E, t), *er = ROW(R, r), *w = ROW(W, r);
    double headSum = 0, tailSum = 0;
    for (int i = 0; i < m->n; i++) {
        headSum += w[i] * eh[i];
        tailSum += w[i] * et[i];
    }
    double energy = 0;
    for (int i = 0; i < m->n; i++)
        energy += fabs(et[i] - tailSum * w[i] - (eh[i] - headSum * w[i]) - er[i]);
    return energy;
}

/* transr/transr.cpp:13-37.  compat: the work vectors persist across calls
 * (never zeroed; transr/trainer.cpp:22-23); fixed: zeroed on every call. */
static double transr_energy(orc_model* m, const double* E, const double* R, const double* W,
                            int h, int t, int r) {
    int n = m->n;
    const double *eh = ROW(E, h), *et = ROW(E, t), *er = ROW(R, r);
    const double* Wr = W + (size_t)r * n * n;
    double *hv = m->hwork, *tv = m->twork;
    if (!m->transr_compat) {
        for (int i = 0; i < n; i++) hv[i] = tv[i] = 0;
    }
    for (int i = 0; i < n; i++) {
        for (int j = 0; j < n; j++) {
            hv[i] += Wr[(size_t)j * n + i] * eh[j];
            tv[i] += Wr[(size_t)j * n + i] * et[j];
        }
    }
    double sum = 0;
    for (int i = 0; i < n; i++) {
        if (m->distance == 0) sum += fabs(tv[i] - hv[i] - er[i]);
        else sum += sqr(tv[i] - hv[i] - er[i]);
    }
    return sum;
}

double orc_triple_energy(orc_model* m, int h, int t, int r) {
    switch (m->model) {
        case ORC_TRANSE: return transe_energy(m, m->ent, m->rel, h, t, r);
        case ORC_TRANSH: return transh_energy(m, m->ent, m->rel, m->w, h, t, r);
        default: return transr_energy(m, m->ent, m->rel, m->w, h, t, r);
    }
}

/* ------------------------------------------------------ gradient updates */

/* transe/trainer.cpp:25-46 */
static void transe_update(orc_model* m, int h, int t, int r, int corrupted) {
    int n = m->n;
    double modifier = corrupted ? 1.0 : -1.0;
    const double *eh = ROW(m->ent, h), *et = ROW(m->ent, t), *er = ROW(m->rel, r);
    double *nr_ = ROW(m->rel_next, r), *nh = ROW(m->ent_next, h), *nt = ROW(m->ent_next, t);
    for (int i = 0; i < n; i++) {
        double x = 2.0 * (et[i] - eh[i] - er[i]);
        if (m->distance == 0) x = x > 0 ? 1 : -1;
        nr_[i] -= modifier * m->lr * x;
        nh[i] -= modifier * m->lr * x;
        nt[i] += modifier * m->lr * x;
    }
    orc_norm(nr_, n, 1);
    orc_norm(nh, n, 1);
    orc_norm(nt, n, 1);
}

/* transh/trainer.cpp:11-59 */
static void transh_update(orc_model* m, int h, int t, int r, int corrupted) {
    int n = m->n;
    double beta = corrupted ? 1 : -1;
    const double *eh = ROW(m->ent, h), *et = ROW(m->ent, t), *er = ROW(m->rel, r), *w = ROW(m->w, r);
    double *nr_ = ROW(m->rel_next, r), *nh = ROW(m->ent_next, h), *nt = ROW(m->ent_next, t);
    double* nw = ROW(m->w_next, r);
    double headSum = 0, tailSum = 0, sum_x = 0;
    for (int i = 0; i < n; i++) {
        headSum += w[i] * eh[i];
        tailSum += w[i] * et[i];
    }
    for (int i = 0; i < n; i++) {
        double x = 2 * (et[i] - tailSum * w[i] - (eh[i] - headSum * w[i]) - er[i]);
        x = x > 0 ? 1 : -1;
        sum_x += x * w[i];
        nr_[i] -= beta * m->lr * x;
        nh[i] -= beta * m->lr * x;
        nt[i] += beta * m->lr * x;
        nw[i] += beta * m->lr * x * headSum;
        nw[i] -= beta * m->lr * x * tailSum;
    }
    for (int i = 0; i < n; i++) {
        nw[i] += beta * m->lr * sum_x * eh[i];
        nw[i] -= beta * m->lr * sum_x * et[i];
    }
    orc_norm(nr_, n, 1);
    orc_norm(nh, n, 1);
    orc_norm(nt, n, 1);
    orc_norm(nw, n, 0);
    g_site = 0; orc_norm_orth(nr_, nw, n, m->lr);
    g_site = 1; orc_norm_orth(nh, nw, n, m->lr);
    g_site = 2; orc_norm_orth(nt, nw, n, m->lr);
    g_site = 3;
}

/* transr/trainer.cpp:144-188 */
static void transr_update(orc_model* m, int h, int t, int r, int corrupted) {
    int n = m->n;
    double beta = corrupted ? 1.0 : -1.0;
    const double *eh = ROW(m->ent, h), *et = ROW(m->ent, t), *er = ROW(m->rel, r);
    const double* W = m->w + (size_t)r * n * n;
    double* Wn = m->w_next + (size_t)r * n * n;
    double *nr_ = ROW(m->rel_next, r), *nh = ROW(m->ent_next, h), *nt = ROW(m->ent_next, t);
    for (int i = 0; i < n; i++) {
        double headSum = 0, tailSum = 0;
        for (int j = 0; j < n; j++) {
            headSum += W[(size_t)j * n + i] * eh[j];
            tailSum += W[(size_t)j * n + i] * et[j];
        }
        double x = 2.0 * (tailSum - headSum - er[i]);
        if (m->distance == 0) x = x > 0 ? 1 : -1;
        for (int j = 0; j < n; j++) {
            Wn[(size_t)j * n + i] -= beta * m->lr * x * (eh[j] - et[j]);
            nh[j] -= beta * m->lr * x * W[(size_t)j * n + i];
            nt[j] += beta * m->lr * x * W[(size_t)j * n + i];
        }
        nr_[i] -= beta * m->lr * x;
    }
    orc_norm(nr_, n, 0);
    orc_norm(nh, n, 0);
    orc_norm(nt, n, 0);
    for (int i = 0; i < n; i++) orc_norm(Wn + (size_t)i * n, n, 0);
    g_site = 0; orc_transr_norm(nh, Wn, n, m->lr);
    g_site = 1; orc_transr_norm(nt, Wn, n, m->lr);
    g_site = 2; orc_transr_norm(ROW(m->ent_next, r), Wn, n, m->lr); /* transr/trainer.cpp:187 (sic) */
    g_site = 3;
}

void orc_gradient_update(orc_model* m, int h, int t, int r, int corrupted) {
    switch (m->model) {
        case ORC_TRANSE: transe_update(m, h, t, r, corrupted); break;
        case ORC_TRANSH: transh_update(m, h, t, r, corrupted); break;
        default: transr_update(m, h, t, r, corrupted); break;
    }
}

/* prebatch: *_next_ = snapshot (transe/trainer.cpp:53-56 and siblings) */
void orc_begin_batch(orc_model* m) {
    size_t n = (size_t)m->n;
    memcpy(m->ent_next, m->ent, sizeof(double) * (size_t)m->ne * n);
    memcpy(m->rel_next, m->rel, sizeof(double) * (size_t)m->nr * n);
    if (m->wsize) memcpy(m->w_next, m->w, sizeof(double) * (size_t)m->wsize);
}

/* postbatch: snapshot = *_next_ (transe/trainer.cpp:48-51 and siblings) */
void orc_end_batch(orc_model* m) {
    double* t;
    t = m->ent; m->ent = m->ent_next; m->ent_next = t;
    t = m->rel; m->rel = m->rel_next; m->rel_next = t;
    t = m->w; m->w = m->w_next; m->w_next = t;
}

/* Trainer::train_kb (common/trainer.cpp:130-149) */
static double train_kb(orc_model* m, int aH, int aT, int aR, int bH, int bT, int bR, long long* active) {
    double loss = 0;
    double normalEnergy = orc_triple_energy(m, aH, aT, aR);
    double corruptedEnergy = orc_triple_energy(m, bH, bT, bR);
    if (normalEnergy + m->margin > corruptedEnergy) {
        loss = m->margin + normalEnergy - corruptedEnergy;
        orc_gradient_update(m, aH, aT, aR, 0);
        orc_gradient_update(m, bH, bT, bR, 1);
        (*active)++;
    }
    return loss;
}

/* The sampling half of Trainer::bfgs (common/trainer.cpp:79-98). */
static void draw_sample(orc_model* m, int* si, int* sj, int* side) {
    int i = orc_randmax(m->ntrain);
    int j = orc_randmax(m->ne);
    int r = m->rels[i];
    double pr = 1000 * m->tail_mean[r] / (m->tail_mean[r] + m->head_mean[r]);
    if (m->method == 0) pr = 500; /* METHOD_UNIF */
    if (orc_rand() % 1000 < pr) {
        while (orc_in_train(m, m->heads[i], r, j)) j = orc_randmax(m->ne);
        *side = 1;
    } else {
        while (orc_in_train(m, j, r, m->tails[i])) j = orc_randmax(m->ne);
        *side = 0;
    }
    *si = i;
    *sj = j;
}

static double run_sample(orc_model* m, int i, int j, int side, long long* active) {
    int h = m->heads[i], t = m->tails[i], r = m->rels[i];
    if (side) return train_kb(m, h, t, r, h, j, r, active);
    return train_kb(m, h, t, r, j, t, r, active);
}

/* Trainer::bfgs, one epoch (common/trainer.cpp:69-107), or a prefix of it. */
double orc_train_batches(orc_model* m, int nbatches, long long* active) {
    int batchsize = m->ntrain / m->nbatches;
    double loss = 0;
    long long act = 0;
    for (int batch = 0; batch < nbatches; batch++) {
        orc_begin_batch(m);
        for (int k = 0; k < batchsize; k++) {
            int i, j, side;
            draw_sample(m, &i, &j, &side);
            loss += run_sample(m, i, j, side, &act);
        }
        orc_end_batch(m);
    }
    if (active) *active = act;
    return loss;
}

double orc_train_epoch(orc_model* m, long long* active) {
    return orc_train_batches(m, m->nbatches, active);
}

double orc_train_replay(orc_model* m, const int* si, const int* sj, const uint8_t* side,
                        long long count, long long* active) {
    int batchsize = m->ntrain / m->nbatches;
    double loss = 0;
    long long act = 0;
    for (long long base = 0; base + batchsize <= count; base += batchsize) {
        orc_begin_batch(m);
        for (int k = 0; k < batchsize; k++)
            loss += run_sample(m, si[base + k], sj[base + k], side[base + k], &act);
        orc_end_batch(m);
    }
    if (active) *active = act;
    return loss;
}

void orc_sample_stream(orc_model* m, long long count, int* si, int* sj, uint8_t* side) {
    for (long long k = 0; k < count; k++) {
        int i, j, s;
        draw_sample(m, &i, &j, &s);
        si[k] = i;
        sj[k] = j;
        side[k] = (uint8_t)s;
    }
}

/* ---------------------------------------------------------- evaluation */

/* EmbeddingEvaluation::run + evalCorruption + cachedTripleEnergy
 * (common/evaluation.cpp:107-251).  For TransR compat the energy work vectors
 * persist over the whole evaluation (transr/evaluation.cpp:22-23), so the cache
 * and the relation-major visit order are reproduced exactly. */
void orc_evaluate(orc_model* m,
                  const int* th, const int* tt, const int* tr, int ntest,
                  const int* fh, const int* ft, const int* fr, int nfilter,
                  double* out) {
    int ne = m->ne;
    uint64_t* keys = (uint64_t*)xcalloc((size_t)nfilter, sizeof(uint64_t));
    for (int k = 0; k < nfilter; k++) keys[k] = fkey(m, fh[k], fr[k], ft[k]);
    qsort(keys, (size_t)nfilter, sizeof(uint64_t), cmp_u64);

    double* cache = NULL;
    if (ne <= 40000) cache = (double*)xcalloc((size_t)ne * ne, sizeof(double)); /* evaluation.h:11 */
    double* energies = (double*)xcalloc((size_t)ne, sizeof(double));
    long long rawSum = 0, filtSum = 0, rawHits = 0, filtHits = 0, ties = 0;

    for (int relationId = 0; relationId < m->nr; relationId++) {
        if (cache)
            for (size_t i = 0; i < (size_t)ne * ne; i++) cache[i] = -1;
        for (int tid = 0; tid < ntest; tid++) {
            if (tr[tid] != relationId) continue;
            int head = th[tid], tail = tt[tid], rel = tr[tid];
            for (int corruptHead = 1; corruptHead >= 0; corruptHead--) {
                for (int i = 0; i < ne; i++) {
                    int ch = corruptHead ? i : head, ct = corruptHead ? tail : i;
                    double e;
                    if (cache) {
                        size_t idx = (size_t)ch * ne + ct;
                        if (cache[idx] >= 0) e = cache[idx];
                        else { e = orc_triple_energy(m, ch, ct, rel); cache[idx] = e; }
                    } else {
                        e = orc_triple_energy(m, ch, ct, rel);
                    }
                    energies[i] = e;
                }
                int truth = corruptHead ? head : tail;
                double et = energies[truth];
                long long raw = 1, filt = 1;
                for (int i = 0; i < ne; i++) {
                    if (i != truth && energies[i] == et) ties++;
                    if (i == truth || !(energies[i] < et)) continue;
                    raw++;
                    int ch = corruptHead ? i : head, ct = corruptHead ? tail : i;
                    if (!filter_has(keys, nfilter, fkey(m, ch, rel, ct))) filt++;
                }
                rawSum += raw;
                filtSum += filt;
                if (raw <= 10) rawHits++;
                if (filt <= 10) filtHits++;
            }
        }
    }
    double numberCorruptions = ntest * 2.0;
    out[0] = rawSum / numberCorruptions;
    out[1] = rawHits / numberCorruptions;
    out[2] = filtSum / numberCorruptions;
    out[3] = filtHits / numberCorruptions;
    out[4] = (double)ties;
    free(cache);
    free(energies);
    free(keys);
}
