// kb2e_cli.cpp -- drop-in command-line front end: trainTransE / trainTransH /
// trainTransR and evalTransE / evalTransH / evalTransR (dispatch on argv[0]).
//
// Same flags, defaults, stdout lines and files as the reference binaries
// (transe/bin/trainTransE.cpp, common/args.cpp, common/loader.cpp,
// common/trainer.cpp:109-127, common/evaluation.cpp:181-266).  The Trainer
// class below keeps the shape of common::Trainer (common/trainer.h:14-78):
// add / loadFiles / train / write, with prepTrain and bfgs as the overridable
// steps -- and bfgs() runs on the GPU through include/kb2e_engine.h.
// GPU-only flags are additive: --precision 64|32, --device N, --transrcompat 0|1,
// --schedule 0|1 (0 = ORDERED, the reference's sequence; 1 = PARALLEL, summed
// per-row deltas with one norm per batch, kb2e_engine.h kb2e_schedule), --gpus N,
// --subbatches K (PARALLEL TransR: each batch applied in K sub-batches).
#include <sys/stat.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <functional>
#include <iostream>
#include <map>
#include <string>
#include <vector>

#include "../../../include/kb2e_engine.h"

namespace kb2e_host {

// ------------------------------------------------------------ arguments

enum { METHOD_UNIF = 0, METHOD_BERN = 1 };
const char* method_name(int m) { return m == METHOD_UNIF ? "unif" : "bern"; }

struct EmbeddingArguments {  // common/args.h:9-25, defaults common/constants.h:28-40
    std::string dataDir = "../data";
    std::string outputDir = ".";
    int embeddingSize = 100;
    double learningRate = 0.001;
    double margin = 1.0;
    int method = METHOD_BERN;
    int numBatches = 100;
    int maxEpochs = 1000;
    int distanceType = 0;
    std::string seedDataDir = ".";
    int seedMethod = METHOD_UNIF;
    unsigned int seed = (unsigned int)time(NULL);
    // GPU engine options (additive)
    int precision = 64;
    int device = 0;
    int transrCompat = 1;
    int schedule = 0;
    int gpus = 1;
    int subBatches = 0;  // 0: the engine's default (kb2e_config.sub_batches)

    std::string to_string() const {  // common/args.cpp:33-50
        std::string r = "Options: [";
        r += "datadir: '" + dataDir + "', ";
        r += "outdir: '" + outputDir + "', ";
        r += "size: " + std::to_string(embeddingSize) + ", ";
        r += "rate: " + std::to_string(learningRate) + ", ";
        r += "margin: " + std::to_string(margin) + ", ";
        r += std::string("method: ") + method_name(method) + ", ";
        r += "batches: " + std::to_string(numBatches) + ", ";
        r += "epochs: " + std::to_string(maxEpochs) + ", ";
        r += "distance: " + std::to_string(distanceType) + ", ";
        r += "seeddatadir: '" + seedDataDir + "', ";
        r += std::string("seedmethod: ") + method_name(seedMethod) + ", ";
        r += "seed: " + std::to_string(seed) + "]";
        return r;
    }
};

// "-flag" or "--flag"; every flag needs a value (common/utils.cpp:55-68).
int argpos(const char* flag, bool hasValue, int argc, char** argv) {
    for (int i = 1; i < argc; i++) {
        if (!strcmp((std::string("-") + flag).c_str(), argv[i]) || !strcmp((std::string("--") + flag).c_str(), argv[i])) {
            if (hasValue && i == argc - 1) {
                printf("Argument missing for %s\n", flag);
                exit(1);
            }
            return i;
        }
    }
    return -1;
}

void printUsage(const char* invoked) {  // common/args.cpp:125-142
    printf("USAGE: %s [option value] ...\n", invoked);
    printf("       %s --help\n", invoked);
    printf("All options require a value.\n");
    printf("Options:\n");
    printf("   --datadir [../data]\n");
    printf("   --outdir [.]\n");
    printf("   --size [100]\n");
    printf("   --rate [0.001000]\n");
    printf("   --margin [1.000000]\n");
    printf("   --method [1 (bern)]\n");
    printf("   --batches [100]\n");
    printf("   --epochs [1000]\n");
    printf("   --distance [0]\n");
    printf("   --seeddatadir [.] (TransR only)\n");
    printf("   --seedmethod [0 (unif)] (TransR only)\n");
    printf("   --seed [now]\n");
    printf("   --precision [64] (GPU: 64 or 32)\n");
    printf("   --device [0] (GPU ordinal)\n");
    printf("   --transrcompat [1] (TransR: reproduce the accumulating energy)\n");
    printf("   --schedule [0] (GPU: 0 ordered = the reference's sequence, 1 parallel)\n");
    printf("   --gpus [1] (GPU: devices --device .. --device+N-1, triples sharded by head, epoch merge over RCCL)\n");
    printf("   --subbatches [engine default] (GPU, parallel TransR: each batch's updates in this many sub-batches)\n");
}

EmbeddingArguments parseArgs(int argc, char** argv) {  // common/args.cpp:53-122
    if (argpos("help", false, argc, argv) != -1) {
        printUsage(argv[0]);
        exit(0);
    }
    EmbeddingArguments a;
    int i;
    if ((i = argpos("datadir", true, argc, argv)) != -1) a.dataDir = argv[i + 1];
    if ((i = argpos("outdir", true, argc, argv)) != -1) a.outputDir = argv[i + 1];
    if ((i = argpos("size", true, argc, argv)) != -1) a.embeddingSize = atoi(argv[i + 1]);
    if ((i = argpos("rate", true, argc, argv)) != -1) a.learningRate = atof(argv[i + 1]);
    if ((i = argpos("margin", true, argc, argv)) != -1) a.margin = atof(argv[i + 1]);
    if ((i = argpos("method", true, argc, argv)) != -1) a.method = atoi(argv[i + 1]);
    if ((i = argpos("batches", true, argc, argv)) != -1) a.numBatches = atoi(argv[i + 1]);
    if ((i = argpos("epochs", true, argc, argv)) != -1) a.maxEpochs = atoi(argv[i + 1]);
    if ((i = argpos("distance", true, argc, argv)) != -1) a.distanceType = atoi(argv[i + 1]);
    if ((i = argpos("seeddatadir", true, argc, argv)) != -1) a.seedDataDir = argv[i + 1];
    if ((i = argpos("seedmethod", true, argc, argv)) != -1) a.seedMethod = atoi(argv[i + 1]);
    if ((i = argpos("seed", true, argc, argv)) != -1) a.seed = atoi(argv[i + 1]);
    if ((i = argpos("precision", true, argc, argv)) != -1) a.precision = atoi(argv[i + 1]);
    if ((i = argpos("device", true, argc, argv)) != -1) a.device = atoi(argv[i + 1]);
    if ((i = argpos("transrcompat", true, argc, argv)) != -1) a.transrCompat = atoi(argv[i + 1]);
    if ((i = argpos("schedule", true, argc, argv)) != -1) a.schedule = atoi(argv[i + 1]) ? 1 : 0;
    if ((i = argpos("gpus", true, argc, argv)) != -1) a.gpus = std::max(1, atoi(argv[i + 1]));
    if ((i = argpos("subbatches", true, argc, argv)) != -1) a.subBatches = std::max(1, atoi(argv[i + 1]));
    return a;
}

bool fileExists(const std::string& path) {
    struct stat b;
    return stat(path.c_str(), &b) == 0;
}

// -------------------------------------------------------------- loader

void loadIdFile(const std::string& path, std::map<std::string, int>& ids) {  // common/loader.cpp:15-24
    FILE* f = fopen(path.c_str(), "r");
    if (!f) {
        printf("Could not open id file: %s\n", path.c_str());
        exit(2);
    }
    char buf[512];
    int id;
    while (fscanf(f, "%511s\t%d", buf, &id) == 2) ids[std::string(buf)] = id;
    fclose(f);
}

void loadTripleFile(const std::string& path, std::map<std::string, int>& ent, std::map<std::string, int>& rel,
                    const std::function<void(int, int, int)>& cb) {  // common/loader.cpp:26-62
    FILE* f = fopen(path.c_str(), "r");
    if (!f) {
        printf("Could not open triple file: %s\n", path.c_str());
        exit(2);
    }
    char hb[512], tb[512], rb[512];
    while (fscanf(f, "%511s\t%511s\t%511s", hb, tb, rb) == 3) {
        bool fail = false;
        if (!ent.count(hb)) {
            std::cout << "Head entity found in triple file that was not found in the identity file: " << hb << std::endl;
            fail = true;
        }
        if (!ent.count(tb)) {
            std::cout << "Tail entity found in triple file that was not found in the identity file: " << tb << std::endl;
            fail = true;
        }
        if (!rel.count(rb)) {
            std::cout << "Relation found in triple file that was not found in the identity file: " << rb << std::endl;
            fail = true;
        }
        if (fail) continue;
        cb(ent[hb], ent[tb], rel[rb]);
    }
    fclose(f);
}

void check(kb2e_ctx* ctx, kb2e_status st, const char* what) {
    if (st != KB2E_OK) {
        printf("kb2e engine error in %s (status %d): %s\n", what, (int)st, ctx ? kb2e_last_error(ctx) : "");
        exit(1);
    }
}

// common/trainer.cpp:109-127: "%.6lf\t" per value, "\n" per row, from the
// device table (formatted on the device).
void writeTable(kb2e_ctx* ctx, int table, const std::string& path) {
    if (kb2e_write_table(ctx, table, path.c_str()) != KB2E_OK) {
        printf("Could not open output file: %s\n", path.c_str());
        exit(1);
    }
}

// transr/trainer.cpp:90-113: the seed file into a device table (parsed on the
// device), with the reference's message when it holds too few numbers.
void readSeed(kb2e_ctx* ctx, int table, const std::string& path, int mode) {
    if (kb2e_read_table(ctx, table, path.c_str(), mode) != KB2E_OK) {
        printf("Failed to read embedding values from seed file: '%s'\n", path.c_str());
        exit(1);
    }
}

// ------------------------------------------------------------- trainer

class Trainer {  // the interface of common::Trainer (common/trainer.h:14-78)
   public:
    Trainer(EmbeddingArguments args, kb2e_model model) : args_(args), model_(model) {}
    virtual ~Trainer() {
        for (kb2e_ctx* c : ranks_) kb2e_destroy(c);
    }

    void add(int head, int tail, int relation) {
        heads_.push_back(head);
        tails_.push_back(tail);
        relations_.push_back(relation);
    }

    void loadFiles() {  // common/trainer.cpp:151-201
        std::map<std::string, int> entity2id, relation2id;
        loadIdFile(args_.dataDir + "/entity2id.txt", entity2id);
        loadIdFile(args_.dataDir + "/relation2id.txt", relation2id);
        loadTripleFile(args_.dataDir + "/train.txt", entity2id, relation2id,
                       [this](int h, int t, int r) { this->add(h, t, r); });
        numRelations_ = (int)relation2id.size();
        numEntities_ = (int)entity2id.size();
        std::cout << "Number of Relations: " << relation2id.size() << std::endl;
        std::cout << "Number of Entities: " << entity2id.size() << std::endl;
    }

    void train() {  // common/trainer.cpp:60-63
        prepTrain();
        if (ranks_.size() > 1)  // rank 0's tables everywhere, the merge's communicator
            check(ctx_, kb2e_comm_init_group(ranks_.data(), (int32_t)ranks_.size()), "comm_init_group");
        bfgs();
    }

    // common/trainer.cpp:109-127: the device tables formatted on the device
    virtual void write() {
        const std::string m = method_name(args_.method);
        writeTable(ctx_, 1, args_.outputDir + "/relation2vec." + m);
        writeTable(ctx_, 0, args_.outputDir + "/entity2vec." + m);
    }

   protected:
    EmbeddingArguments args_;
    kb2e_model model_;
    kb2e_ctx* ctx_ = nullptr;          // rank 0 (the tables write() prints)
    std::vector<kb2e_ctx*> ranks_;     // one context per GPU (--gpus)
    int numRelations_ = 0, numEntities_ = 0;
    std::vector<int> heads_, tails_, relations_;

    // common/trainer.cpp:34-58: the initial tables, drawn from the same
    // glibc stream (seeded with --seed) inside the engine.  --gpus N: one
    // context per device, each training the triples whose head hashes to it
    //  in batches of the single-GPU size (numBatches / N
    // batches an epoch), rank k seeded with seed + k (distinct sample streams;
    // the merge starts every rank from rank 0's tables).
    virtual void prepTrain() {
        const int N = args_.gpus;
        for (int k = 0; k < N; ++k) {
            std::vector<int> h, t, r;
            for (size_t i = 0; i < heads_.size(); ++i)
                if (N == 1 || head_owner(heads_[i], N) == k) {
                    h.push_back(heads_[i]);
                    t.push_back(tails_[i]);
                    r.push_back(relations_[i]);
                }
            ranks_.push_back(make_rank(k, h, t, r));
        }
        ctx_ = ranks_[0];
    }

    // common/trainer.cpp:69-107, on the GPU.
    virtual void bfgs() {
        const int32_t nb = (int32_t)std::max(1, args_.numBatches / args_.gpus);
        for (int epoch = 0; epoch < args_.maxEpochs; epoch++) {
            double loss = 0;
            int64_t active = 0;
            if (ranks_.size() == 1) {
                check(ctx_, kb2e_train_epoch(ctx_, &loss, &active), "train_epoch");
            } else {
                for (kb2e_ctx* c : ranks_) check(c, kb2e_train_batches(c, nb), "train_batches");  // queued
                for (kb2e_ctx* c : ranks_) {
                    double l = 0;
                    int64_t a = 0;
                    check(c, kb2e_take_stats(c, &l, &a), "take_stats");
                    loss += l;
                    active += a;
                }
                check(ctx_, kb2e_merge_epoch_group(ranks_.data(), (int32_t)ranks_.size()), "merge_epoch");
            }
            printf("Epoch: %d, Loss: %f\n", epoch, loss);
            fflush(stdout);
        }
    }

    // the shard owner of a head entity (kb2e_amd/distributed.py shard_heads)
    static int head_owner(int head, int world) {
        const uint64_t h = (uint64_t)(uint32_t)head * 0x9E3779B97F4A7C15ull;
        return (int)((h >> 40) % (uint64_t)world);
    }

    kb2e_ctx* make_rank(int k, const std::vector<int>& h, const std::vector<int>& t, const std::vector<int>& r) {
        kb2e_config cfg;
        kb2e_default_config(&cfg);
        cfg.model = model_;
        cfg.dim = args_.embeddingSize;
        cfg.num_entities = numEntities_;
        cfg.num_relations = numRelations_;
        cfg.learning_rate = args_.learningRate;
        cfg.margin = args_.margin;
        cfg.method = args_.method;
        cfg.distance = args_.distanceType;
        cfg.num_batches = std::max(1, args_.numBatches / args_.gpus);
        cfg.seed = args_.seed + (unsigned)k;
        cfg.precision = args_.precision;
        // KB2E_CLI_ONE_DEVICE=1: every rank on --device (the one-GPU test box; the
        // merge then runs on the engine's local backend instead of RCCL)
        const char* one = getenv("KB2E_CLI_ONE_DEVICE");
        cfg.device = (one && one[0] == '1') ? args_.device : args_.device + k;
        cfg.transr_compat = args_.transrCompat;
        cfg.schedule = args_.schedule ? KB2E_SCHEDULE_PARALLEL : KB2E_SCHEDULE_ORDERED;
        if (args_.subBatches > 0) cfg.sub_batches = args_.subBatches;
        if (h.empty()) {
            printf("kb2e: GPU %d has no training triples (--gpus %d)\n", k, args_.gpus);
            exit(1);
        }
        kb2e_ctx* c = nullptr;
        check(nullptr, kb2e_create(&cfg, &c), "create");
        check(c, kb2e_upload_triples(c, h.data(), t.data(), r.data(), (int64_t)h.size()), "upload_triples");
        // the reference's randn draws and row norms, made on the device from the
        // same stream (kb2e_init_params is the host form of the same thing)
        int64_t ties = 0;
        check(c, kb2e_init_params_device(c, nullptr, nullptr, nullptr, &ties), "init_params");
        if (ties > 0) {
            // an accept/reject decision sat within a few ulps of the density, where
            // the device exp could round unlike glibc's: redo the init on the host
            // (exact) from a fresh context, so the stream position is the reference's
            fprintf(stderr, "kb2e: %lld near-tie randn decisions on the device; initialising on the host\n",
                    (long long)ties);
            kb2e_destroy(c);
            c = nullptr;
            check(nullptr, kb2e_create(&cfg, &c), "create");
            check(c, kb2e_upload_triples(c, h.data(), t.data(), r.data(), (int64_t)h.size()), "upload_triples");
            check(c, kb2e_init_params(c, nullptr, nullptr, nullptr), "init_params");
        }
        return c;
    }
};

class TransHTrainer : public Trainer {  // transh/trainer.cpp:94-105
   public:
    using Trainer::Trainer;
    void write() override {
        Trainer::write();
        writeTable(ctx_, 2, args_.outputDir + "/weights." + method_name(args_.method));
    }
};

class TransRTrainer : public Trainer {
   public:
    using Trainer::Trainer;
    void write() override {  // transr/trainer.cpp:128-142
        Trainer::write();
        writeTable(ctx_, 2, args_.outputDir + "/weights." + method_name(args_.method));
    }

   protected:
    void prepTrain() override {  // transr/trainer.cpp:70-114
        Trainer::prepTrain();
        // seed files parsed on the device; entities unit-normed, relations verbatim
        // (rank 0's tables are broadcast to the other ranks by the merge's init)
        std::string path = args_.seedDataDir + "/entity2vec." + method_name(args_.seedMethod);
        readSeed(ctx_, 0, path, KB2E_READ_UNIT);
        path = args_.seedDataDir + "/relation2vec." + method_name(args_.seedMethod);
        readSeed(ctx_, 1, path, KB2E_READ_VERBATIM);
    }
};

int train_main(int argc, char** argv, kb2e_model model) {
    EmbeddingArguments args = parseArgs(argc, argv);
    printf("%s\n", args.to_string().c_str());
    Trainer* t = model == KB2E_TRANSE ? new Trainer(args, model)
                 : model == KB2E_TRANSH ? (Trainer*)new TransHTrainer(args, model)
                                        : (Trainer*)new TransRTrainer(args, model);
    t->loadFiles();
    t->train();
    t->write();
    delete t;
    return 0;
}

// ------------------------------------------------------------- evaluation

double vec_len(const double* a, int n) {
    double res = 0;
    for (int i = 0; i < n; i++) res += a[i] * a[i];
    return std::sqrt(res);
}

// EmbeddingEvaluation::prepare + run (common/evaluation.cpp:181-266) with the
// ranking on the GPU (kb2e_evaluate; TransR with --transrcompat 1, the default:
// kb2e_evaluate_transr_compat, the reference's stateful energy).
int eval_main(int argc, char** argv, kb2e_model model) {
    EmbeddingArguments args = parseArgs(argc, argv);
    printf("%s\n", args.to_string().c_str());
    const std::string m = method_name(args.method);
    const std::string relPath = args.outputDir + "/relation2vec." + m;
    const std::string entPath = args.outputDir + "/entity2vec." + m;
    const std::string wPath = args.outputDir + "/weights." + m;
    if (!fileExists(relPath)) {
        printf("Could not find relation embedding file: %s. Make sure to specify the path and/or train.\n", relPath.c_str());
        exit(2);
    }
    if (!fileExists(entPath)) {
        printf("Could not find entity embedding file: %s. Make sure to specify the path and/or train.\n", entPath.c_str());
        exit(2);
    }
    std::map<std::string, int> entity2id, relation2id;
    loadIdFile(args.dataDir + "/entity2id.txt", entity2id);
    loadIdFile(args.dataDir + "/relation2id.txt", relation2id);
    const int ne = (int)entity2id.size(), nr = (int)relation2id.size(), n = args.embeddingSize;
    std::vector<int> th, tt, tr, fh, ft, fr;
    auto addFilter = [&](int h, int t, int r) { fh.push_back(h); ft.push_back(t); fr.push_back(r); };
    loadTripleFile(args.dataDir + "/test.txt", entity2id, relation2id, [&](int h, int t, int r) {
        th.push_back(h); tt.push_back(t); tr.push_back(r); addFilter(h, t, r); });
    loadTripleFile(args.dataDir + "/train.txt", entity2id, relation2id, addFilter);
    loadTripleFile(args.dataDir + "/valid.txt", entity2id, relation2id, addFilter);
    if ((model != KB2E_TRANSE) && !fileExists(wPath)) {
        printf("Could not find weight embedding file: %s. Make sure to specify the path and/or train.\n", wPath.c_str());
        exit(2);
    }
    kb2e_config cfg;
    kb2e_default_config(&cfg);
    cfg.model = model;
    cfg.dim = n;
    cfg.num_entities = ne;
    cfg.num_relations = nr;
    cfg.method = args.method;
    cfg.distance = args.distanceType;
    cfg.precision = 64;
    cfg.device = args.device;
    kb2e_ctx* ctx = nullptr;
    check(nullptr, kb2e_create(&cfg, &ctx), "create");
    // the embedding files parsed on the device (EmbeddingEvaluation::loadEmbeddings)
    if (kb2e_read_table(ctx, 1, relPath.c_str(), KB2E_READ_VERBATIM) != KB2E_OK) {
        printf("Failed to read embedding values from file: '%s'\n", relPath.c_str());
        exit(1);
    }
    if (kb2e_read_table(ctx, 0, entPath.c_str(), KB2E_READ_VERBATIM) != KB2E_OK) {
        printf("Failed to read embedding values from file: '%s'\n", entPath.c_str());
        exit(1);
    }
    {
        std::vector<double> E((size_t)ne * n);
        check(ctx, kb2e_download_params(ctx, E.data(), nullptr, nullptr), "download_params");
        for (int i = 0; i < ne; i++) {  // common/evaluation.cpp:99-102
            const double len = vec_len(&E[(size_t)i * n], n);
            if (len - 1 > 1e-3) std::cout << "wrong_entity" << i << ' ' << len << std::endl;
        }
    }
    if (model != KB2E_TRANSE && kb2e_read_table(ctx, 2, wPath.c_str(), KB2E_READ_VERBATIM) != KB2E_OK) {
        printf("Failed to read embedding weight values from seed file: '%s'\n", wPath.c_str());
        exit(1);
    }
    double out[5];
    if (model == KB2E_TRANSR && args.transrCompat) {
        // the reference's evalTransR: energy work vectors accumulate over the
        // whole run (transr/transr.cpp:20-25); progress per relation (:240)
        auto progress = [](double f, void*) {
            printf("\rProcessed %05.2f%% ...", f * 100.0);
            fflush(stdout);
        };
        check(ctx, kb2e_evaluate_transr_compat(ctx, th.data(), tt.data(), tr.data(), (int64_t)th.size(), fh.data(),
                                               ft.data(), fr.data(), (int64_t)fh.size(), nullptr, out, progress,
                                               nullptr), "evaluate");
    } else {
        check(ctx, kb2e_evaluate(ctx, th.data(), tt.data(), tr.data(), (int64_t)th.size(), fh.data(), ft.data(),
                                 fr.data(), (int64_t)fh.size(), out), "evaluate");
        printf("\rProcessed %05.2f%% ...", 100.0);
    }
    printf("\n");
    printf("Raw      -- Rank: %f, Hits@10: %f\n", out[0], out[1]);
    printf("Filtered -- Rank: %f, Hits@10: %f\n", out[2], out[3]);
    kb2e_destroy(ctx);
    return 0;
}

}  // namespace kb2e_host

#ifndef KB2E_CLI_NO_MAIN  // (tests/native/host_check.cpp includes this file for its parser and loader)
int main(int argc, char** argv) {
    std::string prog = argv[0];
    size_t slash = prog.find_last_of('/');
    if (slash != std::string::npos) prog = prog.substr(slash + 1);
    using namespace kb2e_host;
    if (prog == "trainTransE") return train_main(argc, argv, KB2E_TRANSE);
    if (prog == "trainTransH") return train_main(argc, argv, KB2E_TRANSH);
    if (prog == "trainTransR") return train_main(argc, argv, KB2E_TRANSR);
    if (prog == "evalTransE") return eval_main(argc, argv, KB2E_TRANSE);
    if (prog == "evalTransH") return eval_main(argc, argv, KB2E_TRANSH);
    if (prog == "evalTransR") return eval_main(argc, argv, KB2E_TRANSR);
    fprintf(stderr, "invoke as trainTransE|H|R or evalTransE|H|R (got %s)\n", prog.c_str());
    return 2;
}
#endif
