# Build everything in-tree (the built .so files travel to the GPU box with the
# repo snapshot; they are git-ignored).
#   make            libkb2e.so (HIP engine, gfx950) + oracle/liborc.so
#   make ref        also the reference build + fixture harness (needs /root/reference)
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS := --offload-arch=$(ARCH) -O3 -fPIC -std=c++17 -ffp-contract=off -Wall -Iinclude

CSRC := $(filter-out kb2e_amd/csrc/eval.hip kb2e_amd/csrc/textio.hip kb2e_amd/csrc/transr_cons.hip kb2e_amd/csrc/kernels_transr_cons.hpp kb2e_amd/csrc/kernels_transr_wave.hpp kb2e_amd/csrc/kernels_transr_seq.hpp kb2e_amd/csrc/kernels_transr_pipe.hpp kb2e_amd/csrc/kernels_transr_chainw.hpp kb2e_amd/csrc/kernels_transr_chainwp.hpp kb2e_amd/csrc/kernels_transr_chaing.hpp kb2e_amd/csrc/transr_wide.hip kb2e_amd/csrc/kernels_transr_widep.hpp,$(wildcard kb2e_amd/csrc/*.hip kb2e_amd/csrc/*.hpp kb2e_amd/csrc/*.inc)) include/kb2e_engine.h

BINS := bin/trainTransE bin/trainTransH bin/trainTransR bin/evalTransE bin/evalTransH bin/evalTransR

all: kb2e_amd/libkb2e.so bin/kb2e $(BINS) oracle bin/textio_check

bin/kb2e: kb2e_amd/csrc/host/kb2e_cli.cpp include/kb2e_engine.h kb2e_amd/libkb2e.so
	@mkdir -p bin
	g++ -O2 -std=c++17 -Wall -Iinclude -o $@ kb2e_amd/csrc/host/kb2e_cli.cpp -Lkb2e_amd -lkb2e \
	    -Wl,-rpath,'$$ORIGIN/../kb2e_amd'

# host check of the shared formatter / parser against glibc (tests/test_textio.py)
bin/textio_check: tests/native/textio_check.cpp kb2e_amd/csrc/textio.hpp
	@mkdir -p bin
	g++ -O2 -std=c++17 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -o $@ tests/native/textio_check.cpp

$(BINS): bin/kb2e
	ln -sf kb2e $@

# three translation units (the training engine, the evaluator, text I/O + device
# init), compiled in parallel
kb2e_amd/build/engine.o: $(CSRC)
	@mkdir -p kb2e_amd/build
	$(HIPCC) $(HIPFLAGS) -c -o $@ kb2e_amd/csrc/engine.hip

kb2e_amd/build/eval.o: kb2e_amd/csrc/eval.hip kb2e_amd/csrc/eval.hpp kb2e_amd/csrc/hip_util.hpp \
		kb2e_amd/csrc/host_data.hpp kb2e_amd/csrc/kernels_common.hpp kb2e_amd/csrc/kernels_sampler.hpp
	@mkdir -p kb2e_amd/build
	$(HIPCC) $(HIPFLAGS) -c -o $@ kb2e_amd/csrc/eval.hip

kb2e_amd/build/textio.o: kb2e_amd/csrc/textio.hip kb2e_amd/csrc/textio.hpp kb2e_amd/csrc/hip_util.hpp \
		kb2e_amd/csrc/kernels_glibc.hpp kb2e_amd/csrc/glibc_rand.hpp
	@mkdir -p kb2e_amd/build
	$(HIPCC) $(HIPFLAGS) -c -o $@ kb2e_amd/csrc/textio.hip

kb2e_amd/build/transr_cons.o: kb2e_amd/csrc/transr_cons.hip kb2e_amd/csrc/transr_cons.hpp \
		kb2e_amd/csrc/kernels_transr_cons.hpp kb2e_amd/csrc/kernels_transr_wave.hpp kb2e_amd/csrc/kernels_transr_seq.hpp \
		kb2e_amd/csrc/kernels_transr_pipe.hpp kb2e_amd/csrc/kernels_transr_mfma.hpp \
		kb2e_amd/csrc/kernels_transr_chainw.hpp kb2e_amd/csrc/kernels_transr_chainwp.hpp \
		kb2e_amd/csrc/kernels_transr_chaing.hpp \
		kb2e_amd/csrc/kernels_transr_parallel.hpp kb2e_amd/csrc/kernels_common.hpp kb2e_amd/csrc/hip_util.hpp
	@mkdir -p kb2e_amd/build
	$(HIPCC) $(HIPFLAGS) -c -o $@ kb2e_amd/csrc/transr_cons.hip

kb2e_amd/build/transr_wide.o: kb2e_amd/csrc/transr_wide.hip kb2e_amd/csrc/transr_cons.hpp \
		kb2e_amd/csrc/kernels_transr_widep.hpp kb2e_amd/csrc/kernels_transr_seq.hpp kb2e_amd/csrc/kernels_transr_mfma.hpp \
		kb2e_amd/csrc/kernels_transr_parallel.hpp kb2e_amd/csrc/kernels_common.hpp kb2e_amd/csrc/hip_util.hpp
	@mkdir -p kb2e_amd/build
	$(HIPCC) $(HIPFLAGS) -c -o $@ kb2e_amd/csrc/transr_wide.hip

kb2e_amd/libkb2e.so: kb2e_amd/build/engine.o kb2e_amd/build/eval.o kb2e_amd/build/textio.o kb2e_amd/build/transr_cons.o \
		kb2e_amd/build/transr_wide.o
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $^ -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

# diagnostic build: per-phase cycle counters in the relation-owner kernels
prof: kb2e_amd/libkb2e_prof.so

kb2e_amd/build/engine_prof.o: $(CSRC)
	@mkdir -p kb2e_amd/build
	$(HIPCC) $(HIPFLAGS) -DKB2E_OWNER_PROF -c -o $@ kb2e_amd/csrc/engine.hip

kb2e_amd/libkb2e_prof.so: kb2e_amd/build/engine_prof.o kb2e_amd/build/eval.o kb2e_amd/build/textio.o \
		kb2e_amd/build/transr_cons.o kb2e_amd/build/transr_wide.o
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $^ -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

oracle:
	$(MAKE) -C oracle all

# The reference-side binding (integration/gpu_trainer.h) compiled against the
# reference's headers and objects (oracle/_ref/common.a, built from
# /root/reference by `make ref`) and libkb2e.so.  Needs /root/reference; the
# binaries travel to the GPU box in bin/binding/.
REF ?= /root/reference
BINDING := bin/binding/trainTransE bin/binding/trainTransH bin/binding/trainTransR

binding: $(BINDING)

bin/binding/train%: integration/train_gpu.cpp integration/gpu_trainer.h include/kb2e_engine.h kb2e_amd/libkb2e.so ref
	@mkdir -p bin/binding
	g++ -O2 -std=c++11 -Wall -I$(REF) -Iinclude -Iintegration \
	    -DKB2E_BINDING_MODEL=$(if $(filter TransE,$*),0,$(if $(filter TransH,$*),1,2)) \
	    -o $@ integration/train_gpu.cpp oracle/_ref/common.a -Lkb2e_amd -lkb2e \
	    -Wl,-rpath,'$$ORIGIN/../../kb2e_amd'

ref:
	$(MAKE) -C oracle ref

# ASan + UBSan builds of the host code.  CPU (tests/test_sanitize.py
# builds the same three itself): the CLI's parser and loader + the host sample
# stream (tests/native/host_check.cpp), the text formatter / parser, the Bloom
# prefilter.  GPU box: libkb2e_san.so, the engine with its host code instrumented
# (-Xarch_host: the device code is not), and the CLI on it (bin/san/train*, eval*),
# run by tools/gpu_sanitize.sh over the golden tiny set (training, the in-process
# two-context merge, the evaluator, the text tables).
SANFLAGS := -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=all
HIPSAN := $(foreach f,-fsanitize=address -fsanitize=undefined -fno-sanitize-recover=all -fno-omit-frame-pointer,-Xarch_host $(f))
CLANGXX := /opt/rocm/lib/llvm/bin/clang++
SANOBJ := kb2e_amd/build/san

sanitize: bin/san/host_check bin/san/textio_check bin/san/bloom_check kb2e_amd/libkb2e_san.so bin/san/kb2e

bin/san/host_check: tests/native/host_check.cpp kb2e_amd/csrc/host/kb2e_cli.cpp kb2e_amd/csrc/host_data.hpp kb2e_amd/libkb2e.so
	@mkdir -p bin/san
	g++ $(SANFLAGS) -std=c++17 -Iinclude -o $@ tests/native/host_check.cpp -Lkb2e_amd -lkb2e -Wl,-rpath,'$$ORIGIN/../../kb2e_amd'

bin/san/textio_check: tests/native/textio_check.cpp kb2e_amd/csrc/textio.hpp
	@mkdir -p bin/san
	g++ $(SANFLAGS) -std=c++17 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -o $@ tests/native/textio_check.cpp

bin/san/bloom_check: tests/native/bloom_check.cpp kb2e_amd/csrc/host_data.hpp
	@mkdir -p bin/san
	g++ $(SANFLAGS) -std=c++17 -Ikb2e_amd/csrc -o $@ tests/native/bloom_check.cpp

$(SANOBJ)/%.o: kb2e_amd/csrc/%.hip $(CSRC)
	@mkdir -p $(SANOBJ)
	$(HIPCC) $(HIPFLAGS) $(HIPSAN) -g -c -o $@ $<

kb2e_amd/libkb2e_san.so: $(SANOBJ)/engine.o $(SANOBJ)/eval.o $(SANOBJ)/textio.o $(SANOBJ)/transr_cons.o \
		$(SANOBJ)/transr_wide.o
	$(HIPCC) $(HIPFLAGS) $(HIPSAN) -shared-libasan -shared -o $@ $^ -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

bin/san/kb2e: kb2e_amd/csrc/host/kb2e_cli.cpp include/kb2e_engine.h kb2e_amd/libkb2e_san.so
	@mkdir -p bin/san
	$(CLANGXX) -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=all -shared-libasan \
	    -std=c++17 -Iinclude -o $@ kb2e_amd/csrc/host/kb2e_cli.cpp -Lkb2e_amd -l:libkb2e_san.so \
	    -Wl,-rpath,'$$ORIGIN/../../kb2e_amd' -Wl,-rpath,$$(dirname $$($(CLANGXX) -print-file-name=libclang_rt.asan-x86_64.so))
	for b in trainTransE trainTransH trainTransR evalTransE evalTransH evalTransR; do ln -sf kb2e bin/san/$$b; done

clean:
	rm -f kb2e_amd/libkb2e.so kb2e_amd/build/*.o bin/kb2e $(BINS) $(BINDING)
	$(MAKE) -C oracle clean

.PHONY: all oracle ref clean prof binding sanitize
