// oracle/ref_harness.cpp -- golden-fixture generator (TEST INFRASTRUCTURE ONLY).
//
// Linked against the reference's own objects (oracle/_ref/common.a, compiled
// from /root/reference by oracle/Makefile).  It subclasses the reference
// trainers to reach their protected hooks and records, without changing what
// the reference computes:
//   rng    : glibc rand()/randMax/randn known answers      (common/utils.cpp)
//   kat    : energies, norms, orthogonality, transRNorm, single gradient steps
//   train  : a full reference training run on a small dataset: init tables,
//            the exact sample stream, per-sample energies, per-epoch loss and
//            hinge-active counts, per-epoch tables (full precision), and the
//            reference's own text outputs via Trainer::write().
// Output: little-endian .npy files.  Driven by tests/golden/make_golden.py.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "common/args.h"
#include "common/trainer.h"
#include "common/utils.h"
#include "transe/trainer.h"
#include "transe/transe.h"
#include "transh/trainer.h"
#include "transh/transh.h"
#include "transr/trainer.h"
#include "transr/transr.h"

namespace {

std::string g_out;

void write_npy(const std::string& name, const char* descr, size_t esize, const void* data,
               const std::vector<size_t>& shape) {
    std::string dict = std::string("{'descr': '") + descr + "', 'fortran_order': False, 'shape': (";
    for (size_t k = 0; k < shape.size(); k++) {
        dict += std::to_string(shape[k]);
        if (shape.size() == 1 || k + 1 < shape.size()) dict += ",";
        if (k + 1 < shape.size()) dict += " ";
    }
    dict += "), }";
    size_t total = 10 + dict.size() + 1;
    size_t pad = (64 - total % 64) % 64;
    dict += std::string(pad, ' ') + "\n";
    uint16_t hlen = (uint16_t)dict.size();
    FILE* f = fopen((g_out + "/" + name).c_str(), "wb");
    if (!f) { perror(name.c_str()); exit(3); }
    fwrite("\x93NUMPY\x01\x00", 1, 8, f);
    fwrite(&hlen, 2, 1, f);
    fwrite(dict.data(), 1, dict.size(), f);
    size_t count = 1;
    for (size_t s : shape) count *= s;
    fwrite(data, esize, count, f);
    fclose(f);
}

void npy_f64(const std::string& name, const std::vector<double>& v, std::vector<size_t> shape) {
    write_npy(name, "<f8", 8, v.data(), shape);
}
void npy_i64(const std::string& name, const std::vector<long long>& v, std::vector<size_t> shape) {
    write_npy(name, "<i8", 8, v.data(), shape);
}
void npy_i32(const std::string& name, const std::vector<int>& v, std::vector<size_t> shape) {
    write_npy(name, "<i4", 4, v.data(), shape);
}

std::vector<double> flat(const std::vector<std::vector<double>>& t) {
    std::vector<double> out;
    for (auto& r : t) out.insert(out.end(), r.begin(), r.end());
    return out;
}
std::vector<double> flat3(const std::vector<std::vector<std::vector<double>>>& t) {
    std::vector<double> out;
    for (auto& m : t) for (auto& r : m) out.insert(out.end(), r.begin(), r.end());
    return out;
}

// ------------------------------------------------------------------ probes

// Shared recording state for all three models.
struct Recorder {
    std::vector<int> calls;         // (h, t, r) per tripleEnergy call
    std::vector<double> energies;   // value returned per call
    long long updates = 0;          // gradientUpdate calls
    int batches = 0;
    int epoch = 0;
    std::vector<double> epochLoss;
    std::vector<long long> epochActive;
    size_t epochFirstCall = 0;
    long long epochFirstUpdate = 0;
    double margin = 0;
    int recordSampleEpochs = 1;

    void closeEpoch() {
        double loss = 0;
        // train_kb (common/trainer.cpp:130-149): same formula, same order.
        for (size_t c = epochFirstCall; c + 1 < energies.size(); c += 2) {
            double normalEnergy = energies[c], corruptedEnergy = energies[c + 1];
            if (normalEnergy + margin > corruptedEnergy) loss += margin + normalEnergy - corruptedEnergy;
        }
        epochLoss.push_back(loss);
        epochActive.push_back((updates - epochFirstUpdate) / 2);
        epochFirstCall = energies.size();
        epochFirstUpdate = updates;
    }
};

template <class Base>
class Probe : public Base {
   public:
    explicit Probe(common::EmbeddingArguments a) : Base(a) {}
    Recorder rec;
    bool transrFixed = false;

    // -- accessors for the protected reference state
    int ne() { return this->numEntities_; }
    int nr() { return this->numRelations_; }
    int n() { return this->embeddingSize_; }
    std::vector<std::vector<double>>& ent() { return this->entityVec_; }
    std::vector<std::vector<double>>& rel() { return this->relationVec_; }
    void setMargin() { rec.margin = this->margin_; }

    void dumpTables(const std::string& prefix);

   protected:
    void prepTrain() override {
        Base::prepTrain();
        dumpTables("init_");
    }
    double tripleEnergy(int h, int t, int r) override;
    void gradientUpdate(int h, int t, int r, bool corrupted) override {
        rec.updates++;
        Base::gradientUpdate(h, t, r, corrupted);
    }
    void postbatch() override {
        Base::postbatch();
        rec.batches++;
        if (rec.batches % this->numBatches_ == 0) {
            rec.closeEpoch();
            dumpTables("epoch" + std::to_string(rec.epoch) + "_");
            rec.epoch++;
        }
    }
};

template <class Base>
double Probe<Base>::tripleEnergy(int h, int t, int r) {
    double e = Base::tripleEnergy(h, t, r);
    rec.calls.push_back(h);
    rec.calls.push_back(t);
    rec.calls.push_back(r);
    rec.energies.push_back(e);
    return e;
}

// TransR "fixed" energy: the same reference function with the persistent work
// vectors zeroed before each call (the one-line fix of transr/transr.cpp:20-25).
template <>
double Probe<transr::Trainer>::tripleEnergy(int h, int t, int r) {
    if (transrFixed) {
        std::fill(headWorkVec_.begin(), headWorkVec_.end(), 0.0);
        std::fill(tailWorkVec_.begin(), tailWorkVec_.end(), 0.0);
    }
    double e = transr::Trainer::tripleEnergy(h, t, r);
    rec.calls.push_back(h);
    rec.calls.push_back(t);
    rec.calls.push_back(r);
    rec.energies.push_back(e);
    return e;
}

template <>
void Probe<transe::Trainer>::dumpTables(const std::string& p) {
    npy_f64(p + "ent.npy", flat(entityVec_), {(size_t)numEntities_, (size_t)embeddingSize_});
    npy_f64(p + "rel.npy", flat(relationVec_), {(size_t)numRelations_, (size_t)embeddingSize_});
}
template <>
void Probe<transh::Trainer>::dumpTables(const std::string& p) {
    npy_f64(p + "ent.npy", flat(entityVec_), {(size_t)numEntities_, (size_t)embeddingSize_});
    npy_f64(p + "rel.npy", flat(relationVec_), {(size_t)numRelations_, (size_t)embeddingSize_});
    npy_f64(p + "w.npy", flat(weights_), {(size_t)numRelations_, (size_t)embeddingSize_});
}
template <>
void Probe<transr::Trainer>::dumpTables(const std::string& p) {
    npy_f64(p + "ent.npy", flat(entityVec_), {(size_t)numEntities_, (size_t)embeddingSize_});
    npy_f64(p + "rel.npy", flat(relationVec_), {(size_t)numRelations_, (size_t)embeddingSize_});
    npy_f64(p + "w.npy", flat3(weights_),
            {(size_t)numRelations_, (size_t)embeddingSize_, (size_t)embeddingSize_});
    npy_f64(p + "hwork.npy", headWorkVec_, {(size_t)embeddingSize_});
    npy_f64(p + "twork.npy", tailWorkVec_, {(size_t)embeddingSize_});
}

template <class T>
int run_train(common::EmbeddingArguments args, bool transrFixed) {
    srand(args.seed);  // trainTransE.cpp:13
    Probe<T>* trainer = new Probe<T>(args);
    trainer->transrFixed = transrFixed;
    trainer->setMargin();
    trainer->loadFiles();
    trainer->train();
    trainer->write();
    Recorder& rec = trainer->rec;
    npy_f64("epoch_loss.npy", rec.epochLoss, {rec.epochLoss.size()});
    npy_i64("epoch_active.npy", rec.epochActive, {rec.epochActive.size()});
    size_t ncalls = rec.energies.size();
    npy_i32("calls.npy", rec.calls, {ncalls, 3});
    npy_f64("energies.npy", rec.energies, {ncalls});
    // The next rand() values after training, to pin RNG consumption.
    std::vector<int> after;
    for (int k = 0; k < 8; k++) after.push_back(std::rand());
    npy_i32("rand_after.npy", after, {after.size()});
    delete trainer;
    return 0;
}

// ------------------------------------------------------------------- rng

int run_rng() {
    std::vector<int> seeds = {0, 1, 7, 42, 12345, 2147483647};
    std::vector<int> raw;
    for (int s : seeds) {
        srand((unsigned)s);
        for (int k = 0; k < 1000; k++) raw.push_back(std::rand());
    }
    npy_i32("rng_seeds.npy", seeds, {seeds.size()});
    npy_i32("rng_raw.npy", raw, {seeds.size(), 1000});
    std::vector<int> bounds = {1, 2, 3, 1000, 14951, 40943, 483142, 1000000, 2147483647};
    std::vector<int> rm;
    srand(7);
    for (int b : bounds)
        for (int k = 0; k < 200; k++) rm.push_back(common::randMax(b));
    npy_i32("randmax_bounds.npy", bounds, {bounds.size()});
    npy_i32("randmax_seed7.npy", rm, {bounds.size(), 200});
    std::vector<double> rn;
    srand(11);
    for (int k = 0; k < 500; k++) rn.push_back(common::randn(0, 1.0 / 100, -6 / std::sqrt(100), 6 / std::sqrt(100)));
    for (int k = 0; k < 500; k++) rn.push_back(common::randn(0, 1.0 / 50, -1, 1));
    npy_f64("randn_seed11.npy", rn, {2, 500});
    std::vector<int> after;
    for (int k = 0; k < 4; k++) after.push_back(std::rand());
    npy_i32("randn_seed11_after.npy", after, {after.size()});
    return 0;
}

// ------------------------------------------------------------------- kat

double u(double lo, double hi) { return lo + (hi - lo) * (std::rand() / (RAND_MAX + 1.0)); }

std::vector<std::vector<double>> table(int rows, int n, double lo, double hi) {
    std::vector<std::vector<double>> t(rows, std::vector<double>(n));
    for (auto& r : t) for (auto& x : r) x = u(lo, hi);
    return t;
}

template <class T>
class KatProbe : public T {
   public:
    explicit KatProbe(common::EmbeddingArguments a) : T(a) {}
    using T::entityVec_;
    using T::relationVec_;
    using T::numEntities_;
    using T::numRelations_;
    using T::prebatch;
    using T::postbatch;
    using T::gradientUpdate;
};

class TransRKat : public transr::Trainer {
   public:
    explicit TransRKat(common::EmbeddingArguments a) : transr::Trainer(a) {}
    using transr::Trainer::transRNorm;
    using transr::Trainer::weights_;
    using transr::Trainer::weights_next_;
    using transr::Trainer::entityVec_next_;
    using transr::Trainer::relationVec_next_;
    using transr::Trainer::entityVec_;
    using transr::Trainer::relationVec_;
    using transr::Trainer::numEntities_;
    using transr::Trainer::numRelations_;
    using transr::Trainer::prebatch;
    using transr::Trainer::postbatch;
    using transr::Trainer::gradientUpdate;
    using transr::Trainer::headWorkVec_;
    using transr::Trainer::tailWorkVec_;
};

class TransHKat : public transh::Trainer {
   public:
    explicit TransHKat(common::EmbeddingArguments a) : transh::Trainer(a) {}
    using transh::Trainer::weights_;
    using transh::Trainer::weights_next_;
    using transh::Trainer::entityVec_next_;
    using transh::Trainer::relationVec_next_;
    using transh::Trainer::entityVec_;
    using transh::Trainer::relationVec_;
    using transh::Trainer::numEntities_;
    using transh::Trainer::numRelations_;
    using transh::Trainer::prebatch;
    using transh::Trainer::postbatch;
    using transh::Trainer::gradientUpdate;
};

class TransEKat : public transe::Trainer {
   public:
    explicit TransEKat(common::EmbeddingArguments a) : transe::Trainer(a) {}
    using transe::Trainer::entityVec_next_;
    using transe::Trainer::relationVec_next_;
    using transe::Trainer::entityVec_;
    using transe::Trainer::relationVec_;
    using transe::Trainer::numEntities_;
    using transe::Trainer::numRelations_;
    using transe::Trainer::prebatch;
    using transe::Trainer::postbatch;
    using transe::Trainer::gradientUpdate;
};

int run_kat() {
    srand(2024);
    const int n = 16, NE = 12, NR = 4;
    // -- common::norm / norm(a,b,rate)
    {
        std::vector<double> in, out;
        for (int c = 0; c < 64; c++) {
            double scale = (c % 4 == 0) ? 0.05 : (c % 4 == 1 ? 0.3 : (c % 4 == 2 ? 1.0 : 3.0));
            std::vector<double> a(n);
            for (auto& x : a) x = u(-scale, scale);
            in.insert(in.end(), a.begin(), a.end());
            std::vector<double> b1 = a, b2 = a;
            common::norm(b1);
            common::norm(b2, false);
            out.insert(out.end(), b1.begin(), b1.end());
            out.insert(out.end(), b2.begin(), b2.end());
        }
        npy_f64("norm_in.npy", in, {64, (size_t)n});
        npy_f64("norm_out.npy", out, {64, 2, (size_t)n});
    }
    {
        std::vector<double> ain, bin, aout, bout;
        for (int c = 0; c < 64; c++) {
            std::vector<double> a(n), b(n);
            for (auto& x : b) x = u(-1, 1);
            // half the cases are aligned so that b.a > 0.1 and the loop iterates
            for (int i = 0; i < n; i++) a[i] = (c % 2 == 0) ? b[i] * u(0.2, 1.0) : u(-0.3, 0.3);
            double rate = (c % 3 == 0) ? 0.001 : (c % 3 == 1 ? 0.05 : 0.3);
            ain.insert(ain.end(), a.begin(), a.end());
            bin.insert(bin.end(), b.begin(), b.end());
            bin.push_back(rate);
            common::norm(a, b, rate);
            aout.insert(aout.end(), a.begin(), a.end());
            bout.insert(bout.end(), b.begin(), b.end());
        }
        npy_f64("orth_a_in.npy", ain, {64, (size_t)n});
        npy_f64("orth_b_in.npy", bin, {64, (size_t)n + 1});
        npy_f64("orth_a_out.npy", aout, {64, (size_t)n});
        npy_f64("orth_b_out.npy", bout, {64, (size_t)n});
    }
    // -- energies (free functions) on random tables
    common::EmbeddingArguments args;
    args.embeddingSize = n;
    args.learningRate = 0.01;
    args.margin = 1.0;
    args.numBatches = 1;
    auto E = table(NE, n, -0.5, 0.5);
    auto R = table(NR, n, -0.5, 0.5);
    auto Wh = table(NR, n, -1, 1);
    for (auto& w : Wh) common::norm(w, false);
    std::vector<std::vector<std::vector<double>>> Wr(NR, table(n, n, -0.3, 0.3));
    for (int r = 0; r < NR; r++) Wr[r] = table(n, n, -0.3, 0.3);
    npy_f64("kat_E.npy", flat(E), {(size_t)NE, (size_t)n});
    npy_f64("kat_R.npy", flat(R), {(size_t)NR, (size_t)n});
    npy_f64("kat_Wh.npy", flat(Wh), {(size_t)NR, (size_t)n});
    npy_f64("kat_Wr.npy", flat3(Wr), {(size_t)NR, (size_t)n, (size_t)n});
    std::vector<int> trip;
    for (int c = 0; c < 40; c++) {
        trip.push_back(std::rand() % NE);
        trip.push_back(c % 7 == 0 ? trip[trip.size() - 1] : std::rand() % NE);  // some h == t
        trip.push_back(std::rand() % NR);
    }
    npy_i32("kat_triples.npy", trip, {40, 3});
    std::vector<double> eE1, eE2, eH, eR1, eRacc;
    std::vector<double> hv(n, 0.0), tv(n, 0.0);
    for (int c = 0; c < 40; c++) {
        int h = trip[3 * c], t = trip[3 * c + 1], r = trip[3 * c + 2];
        eE1.push_back(transe::tripleEnergy(h, t, r, n, E, R, true));
        eE2.push_back(transe::tripleEnergy(h, t, r, n, E, R, false));
        eH.push_back(transh::tripleEnergy(h, t, r, n, E, R, Wh));
        std::vector<double> z1(n, 0.0), z2(n, 0.0);
        eR1.push_back(transr::tripleEnergy(h, t, r, n, E, R, Wr, 0, z1, z2));
        // accumulating work vectors, as the reference trainer/evaluator use them
        eRacc.push_back(transr::tripleEnergy(h, t, r, n, E, R, Wr, 0, hv, tv));
    }
    npy_f64("kat_energy_transe_l1.npy", eE1, {40});
    npy_f64("kat_energy_transe_l2.npy", eE2, {40});
    npy_f64("kat_energy_transh.npy", eH, {40});
    npy_f64("kat_energy_transr_fresh.npy", eR1, {40});
    npy_f64("kat_energy_transr_accum.npy", eRacc, {40});

    // -- transRNorm (protected member) through a subclass
    {
        args.numBatches = 1;
        TransRKat tr(args);
        std::vector<double> ain, bin, aout, bout;
        for (int c = 0; c < 24; c++) {
            std::vector<double> a(n);
            double s = (c % 2 == 0) ? 0.9 : 0.2;
            for (auto& x : a) x = u(-s, s);
            auto b = table(n, n, -0.5, 0.5);
            ain.insert(ain.end(), a.begin(), a.end());
            auto fb = flat(b);
            bin.insert(bin.end(), fb.begin(), fb.end());
            tr.transRNorm(a, b);
            aout.insert(aout.end(), a.begin(), a.end());
            auto fo = flat(b);
            bout.insert(bout.end(), fo.begin(), fo.end());
        }
        npy_f64("transrnorm_a_in.npy", ain, {24, (size_t)n});
        npy_f64("transrnorm_b_in.npy", bin, {24, (size_t)n, (size_t)n});
        npy_f64("transrnorm_a_out.npy", aout, {24, (size_t)n});
        npy_f64("transrnorm_b_out.npy", bout, {24, (size_t)n, (size_t)n});
    }

    // -- single gradient steps: prebatch, gradientUpdate(pos), gradientUpdate(neg), read next
    for (int distance = 0; distance < 2; distance++) {
        args.distanceType = distance;
        TransEKat te(args);
        te.entityVec_ = E;
        te.relationVec_ = R;
        te.numEntities_ = NE;
        te.numRelations_ = NR;
        std::vector<double> ent, rel;
        for (int c = 0; c < 8; c++) {
            te.prebatch();
            int h = trip[3 * c], t = trip[3 * c + 1], r = trip[3 * c + 2];
            te.gradientUpdate(h, t, r, false);
            te.gradientUpdate((h + 1) % NE, t, r, true);
            auto fe = flat(te.entityVec_next_), fr = flat(te.relationVec_next_);
            ent.insert(ent.end(), fe.begin(), fe.end());
            rel.insert(rel.end(), fr.begin(), fr.end());
        }
        std::string p = distance == 0 ? "step_transe_l1_" : "step_transe_l2_";
        npy_f64(p + "ent.npy", ent, {8, (size_t)NE, (size_t)n});
        npy_f64(p + "rel.npy", rel, {8, (size_t)NR, (size_t)n});
    }
    {
        args.distanceType = 0;
        TransHKat th(args);
        th.entityVec_ = E;
        th.relationVec_ = R;
        th.weights_ = Wh;
        th.numEntities_ = NE;
        th.numRelations_ = NR;
        std::vector<double> ent, rel, w;
        for (int c = 0; c < 8; c++) {
            th.prebatch();
            int h = trip[3 * c], t = trip[3 * c + 1], r = trip[3 * c + 2];
            th.gradientUpdate(h, t, r, false);
            th.gradientUpdate(h, (t + 3) % NE, r, true);
            auto fe = flat(th.entityVec_next_), fr = flat(th.relationVec_next_), fw = flat(th.weights_next_);
            ent.insert(ent.end(), fe.begin(), fe.end());
            rel.insert(rel.end(), fr.begin(), fr.end());
            w.insert(w.end(), fw.begin(), fw.end());
        }
        npy_f64("step_transh_ent.npy", ent, {8, (size_t)NE, (size_t)n});
        npy_f64("step_transh_rel.npy", rel, {8, (size_t)NR, (size_t)n});
        npy_f64("step_transh_w.npy", w, {8, (size_t)NR, (size_t)n});
    }
    for (int distance = 0; distance < 2; distance++) {
        args.distanceType = distance;
        TransRKat trk(args);
        trk.entityVec_ = E;
        trk.relationVec_ = R;
        trk.weights_ = Wr;
        trk.numEntities_ = NE;
        trk.numRelations_ = NR;
        std::vector<double> ent, rel, w;
        for (int c = 0; c < 8; c++) {
            trk.prebatch();
            int h = trip[3 * c], t = trip[3 * c + 1], r = trip[3 * c + 2];
            trk.gradientUpdate(h, t, r, false);
            trk.gradientUpdate(h, (t + 5) % NE, r, true);
            auto fe = flat(trk.entityVec_next_), fr = flat(trk.relationVec_next_);
            auto fw = flat3(trk.weights_next_);
            ent.insert(ent.end(), fe.begin(), fe.end());
            rel.insert(rel.end(), fr.begin(), fr.end());
            w.insert(w.end(), fw.begin(), fw.end());
        }
        std::string p = distance == 0 ? "step_transr_l1_" : "step_transr_l2_";
        npy_f64(p + "ent.npy", ent, {8, (size_t)NE, (size_t)n});
        npy_f64(p + "rel.npy", rel, {8, (size_t)NR, (size_t)n});
        npy_f64(p + "w.npy", w, {8, (size_t)NR, (size_t)n, (size_t)n});
    }
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: ref_harness rng|kat <outdir>\n"
                        "       ref_harness train <E|H|R> <outdir> [fixed] -- <reference trainer flags>\n");
        return 2;
    }
    std::string mode = argv[1];
    g_out = argv[2];
    if (mode == "rng") return run_rng();
    if (mode == "kat") return run_kat();
    if (mode == "train" && argc >= 4) {
        g_out = argv[3];
        std::string model = argv[2];
        int k = 4;
        bool fixed = false;
        if (k < argc && std::string(argv[k]) == "fixed") { fixed = true; k++; }
        if (k < argc && std::string(argv[k]) == "--") k++;
        // parseArgs skips argv[0]; hand it the remaining flags.
        std::vector<char*> av;
        av.push_back(argv[0]);
        for (int q = k; q < argc; q++) av.push_back(argv[q]);
        common::EmbeddingArguments args = common::parseArgs((int)av.size(), av.data());
        args.outputDir = g_out;
        printf("%s\n", args.to_string().c_str());
        if (model == "E") return run_train<transe::Trainer>(args, false);
        if (model == "H") return run_train<transh::Trainer>(args, false);
        if (model == "R") return run_train<transr::Trainer>(args, fixed);
    }
    fprintf(stderr, "bad arguments\n");
    return 2;
}
