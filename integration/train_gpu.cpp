// train_gpu.cpp -- trainTransE/H/R mains on the GPU binding: the reference's
// main (transe/bin/trainTransE.cpp:9-20, transh/bin/trainTransH.cpp,
// transr/bin/trainTransR.cpp) with the model trainer swapped for
// kb2e_binding::GpuTrainer.  Built three times by `make binding`
// (-DKB2E_BINDING_MODEL=0/1/2).
#include <cstdio>
#include <cstdlib>

#include "common/args.h"
#include "gpu_trainer.h"
#include "transe/trainer.h"
#include "transh/trainer.h"
#include "transr/trainer.h"

#if KB2E_BINDING_MODEL == 0
using Trainer = kb2e_binding::GpuTrainer<transe::Trainer, KB2E_TRANSE>;
#elif KB2E_BINDING_MODEL == 1
using Trainer = kb2e_binding::GpuTrainer<transh::Trainer, KB2E_TRANSH>;
#else
using Trainer = kb2e_binding::GpuTrainer<transr::Trainer, KB2E_TRANSR>;
#endif

int main(int argc, char** argv) {
    common::EmbeddingArguments args = common::parseArgs(argc, argv);
    printf("%s\n", args.to_string().c_str());
    srand(args.seed);  // the host init draws (prepTrain) come from this stream
    Trainer* trainer = new Trainer(args);
    trainer->loadFiles();
    trainer->train();
    trainer->write();
    delete trainer;
    return 0;
}
