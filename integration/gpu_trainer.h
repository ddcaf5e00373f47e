// gpu_trainer.h -- the reference-side binding: a drop-in subclass of the
// reference's model trainers (transe/trainer.h:12-28, transh/trainer.h:11-30,
// transr/trainer.h:12-46) whose bfgs() (common/trainer.h:59, the loop of
// common/trainer.cpp:69-107) runs on the kb2e_amd MI355X engine through the C
// ABI of include/kb2e_engine.h.  Everything else -- argument parsing, loadFiles,
// prepTrain's initialisation and TransR seed reading, write() -- is the
// reference's own code, unchanged.
//
// A maintainer adds this header to the reference tree and constructs
// kb2e_binding::GpuTrainer<transe::Trainer, KB2E_TRANSE> in trainTransE's main
// (integration/train_gpu.cpp shows the three mains).  Compiled here against
// /root/reference's headers and oracle/_ref/common.a (the reference's objects)
// by `make binding`; tests/test_gpu_binding.py runs it.
//
// Engine options the reference's parser has no flag for come from the
// environment: KB2E_SCHEDULE (0 ordered = the reference's semantics, default;
// 1 parallel), KB2E_PRECISION (64 default, 32), KB2E_DEVICE, KB2E_TRANSR_FIXED.
#ifndef KB2E_BINDING_GPU_TRAINER_H_
#define KB2E_BINDING_GPU_TRAINER_H_

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

#include "common/args.h"
#include "common/trainer.h"
#include "kb2e_engine.h"

namespace kb2e_binding {

inline int env_int(const char* name, int dflt) {
    const char* v = std::getenv(name);
    return v && *v ? std::atoi(v) : dflt;
}

template <class Base, kb2e_model M>
class GpuTrainer final : public Base {
   public:
    explicit GpuTrainer(common::EmbeddingArguments args)
        : Base(args), seed_(args.seed), distance_(args.distanceType) {}
    // common::Trainer has no virtual destructor: main deletes through this type.
    ~GpuTrainer() { release(); }

   protected:
    // The reference's own prepTrain (sizes the tables, draws the init values from
    // the global rand() stream srand(seed) in main started, TransR: identity Mr
    // and the seed files, common/trainer.cpp:34-58, transh/trainer.cpp:77-88,
    // transr/trainer.cpp:70-113), then the same state on the device.
    void prepTrain() override {
        Base::prepTrain();
        kb2e_config c;
        kb2e_default_config(&c);
        c.model = M;
        c.dim = this->embeddingSize_;
        c.num_entities = this->numEntities_;
        c.num_relations = this->numRelations_;
        c.learning_rate = this->learningRate_;
        c.margin = this->margin_;
        c.method = this->method_;
        c.distance = distance_;
        c.num_batches = this->numBatches_;
        c.seed = seed_;
        c.precision = env_int("KB2E_PRECISION", 64);
        c.schedule = env_int("KB2E_SCHEDULE", KB2E_SCHEDULE_ORDERED);
        c.device = env_int("KB2E_DEVICE", 0);
        c.transr_compat = env_int("KB2E_TRANSR_FIXED", 0) ? 0 : 1;
        c.sub_batches = env_int("KB2E_SUB_BATCHES", c.sub_batches);  // PARALLEL TransR only
        check(kb2e_create(&c, &ctx_), "kb2e_create");
        const int64_t n = (int64_t)this->heads_.size();
        check(kb2e_upload_triples(ctx_, this->heads_.data(), this->tails_.data(), this->relations_.data(), n),
              "kb2e_upload_triples");
        // The engine's own glibc stream (seeded like srand(seed)) draws the same
        // init values, which leaves it where the reference's stream is when
        // bfgs() starts sampling; the host tables must agree bit for bit.
        std::vector<double> e, r, w;
        alloc(e, r, w);
        check(kb2e_init_params(ctx_, e.data(), r.data(), w.empty() ? nullptr : w.data()), "kb2e_init_params");
        if (M != KB2E_TRANSR) {  // TransR overwrote its draws with the seed files
            if (!same(e, this->entityVec_) || !same(r, this->relationVec_)) {
                printf("kb2e: device init differs from the reference's init\n");
                exit(1);
            }
        }
        pack(this->entityVec_, e);
        pack(this->relationVec_, r);
        pack_weights(w);
        check(kb2e_upload_params(ctx_, e.data(), r.data(), w.empty() ? nullptr : w.data()), "kb2e_upload_params");
    }

    // common/trainer.cpp:69-107 on the device: one kb2e_train_epoch per epoch,
    // the reference's epoch line, then the tables back into the host vectors
    // that write() prints.
    void bfgs() override {
        for (int epoch = 0; epoch < this->maxEpochs_; epoch++) {
            double loss = 0;
            int64_t active = 0;
            check(kb2e_train_epoch(ctx_, &loss, &active), "kb2e_train_epoch");
            printf("Epoch: %d, Loss: %f\n", epoch, loss);
        }
        std::vector<double> e, r, w;
        alloc(e, r, w);
        check(kb2e_download_params(ctx_, e.data(), r.data(), w.empty() ? nullptr : w.data()),
              "kb2e_download_params");
        unpack(e, this->entityVec_);
        unpack(r, this->relationVec_);
        unpack_weights(w);
        release();
    }

   private:
    unsigned int seed_;
    int distance_;  // --distance (TransH ignores it, as the reference does)
    kb2e_ctx* ctx_ = nullptr;

    void release() {
        if (ctx_) kb2e_destroy(ctx_);
        ctx_ = nullptr;
    }

    void check(kb2e_status s, const char* what) {
        if (s != KB2E_OK) {  // the reference's convention: message + exit(1)
            printf("%s failed: %s\n", what, ctx_ ? kb2e_last_error(ctx_) : "no engine");
            exit(1);
        }
    }

    size_t weight_elems() const {
        const size_t n = (size_t)this->embeddingSize_, R = (size_t)this->numRelations_;
        return M == KB2E_TRANSH ? R * n : M == KB2E_TRANSR ? R * n * n : 0;
    }

    void alloc(std::vector<double>& e, std::vector<double>& r, std::vector<double>& w) const {
        e.assign((size_t)this->numEntities_ * this->embeddingSize_, 0.0);
        r.assign((size_t)this->numRelations_ * this->embeddingSize_, 0.0);
        w.assign(weight_elems(), 0.0);
    }

    static void pack(const std::vector<std::vector<double>>& t, std::vector<double>& flat) {
        size_t k = 0;
        for (const auto& row : t)
            for (double v : row) flat[k++] = v;
    }
    static void unpack(const std::vector<double>& flat, std::vector<std::vector<double>>& t) {
        size_t k = 0;
        for (auto& row : t)
            for (double& v : row) v = flat[k++];
    }
    static bool same(const std::vector<double>& flat, const std::vector<std::vector<double>>& t) {
        size_t k = 0;
        for (const auto& row : t)
            for (double v : row)
                if (std::memcmp(&v, &flat[k++], sizeof(double)) != 0) return false;
        return true;
    }

    // TransH: weights_[r][i] (transh/trainer.h:16); TransR: weights_[r][j][i]
    // (transr/trainer.h:31), both row-major in the ABI.  Only the overload for
    // M is instantiated, so TransE (no weights_) compiles.
    void pack_weights(std::vector<double>& w) {
        if (w.empty()) return;
        pack_weights_impl(w, std::integral_constant<int, M>());
    }
    void unpack_weights(const std::vector<double>& w) {
        if (w.empty()) return;
        unpack_weights_impl(w, std::integral_constant<int, M>());
    }
    template <class X> void pack_weights_impl(std::vector<double>&, X) {}
    template <class X> void unpack_weights_impl(const std::vector<double>&, X) {}
    void pack_weights_impl(std::vector<double>& w, std::integral_constant<int, KB2E_TRANSH>) {
        pack(this->weights_, w);
    }
    void unpack_weights_impl(const std::vector<double>& w, std::integral_constant<int, KB2E_TRANSH>) {
        unpack(w, this->weights_);
    }
    void pack_weights_impl(std::vector<double>& w, std::integral_constant<int, KB2E_TRANSR>) {
        size_t k = 0;
        for (const auto& m : this->weights_)
            for (const auto& row : m)
                for (double v : row) w[k++] = v;
    }
    void unpack_weights_impl(const std::vector<double>& w, std::integral_constant<int, KB2E_TRANSR>) {
        size_t k = 0;
        for (auto& m : this->weights_)
            for (auto& row : m)
                for (double& v : row) v = w[k++];
    }
};

}  // namespace kb2e_binding

#endif  // KB2E_BINDING_GPU_TRAINER_H_
