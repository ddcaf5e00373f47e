# Build everything in-tree (the built .so files travel to the GPU box with the
# repo snapshot; they are git-ignored).
#   make            libkb2e.so (HIP engine, gfx950) + oracle/liborc.so
#   make ref        also the reference build + fixture harness (needs /root/reference)
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS := --offload-arch=$(ARCH) -O3 -fPIC -std=c++17 -ffp-contract=off -Wall -Iinclude

CSRC := $(wildcard kb2e_amd/csrc/*.hip kb2e_amd/csrc/*.hpp kb2e_amd/csrc/*.inc) include/kb2e_engine.h

BINS := bin/trainTransE bin/trainTransH bin/trainTransR bin/evalTransE bin/evalTransH bin/evalTransR

all: kb2e_amd/libkb2e.so bin/kb2e $(BINS) oracle

bin/kb2e: kb2e_amd/csrc/host/kb2e_cli.cpp include/kb2e_engine.h kb2e_amd/libkb2e.so
	@mkdir -p bin
	g++ -O2 -std=c++17 -Wall -Iinclude -o $@ kb2e_amd/csrc/host/kb2e_cli.cpp -Lkb2e_amd -lkb2e \
	    -Wl,-rpath,'$$ORIGIN/../kb2e_amd'

$(BINS): bin/kb2e
	ln -sf kb2e $@

kb2e_amd/libkb2e.so: $(CSRC)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ kb2e_amd/csrc/engine.hip

# diagnostic build: per-phase cycle counters in the relation-owner kernels
prof: kb2e_amd/libkb2e_prof.so

kb2e_amd/libkb2e_prof.so: $(CSRC)
	$(HIPCC) $(HIPFLAGS) -DKB2E_OWNER_PROF -shared -o $@ kb2e_amd/csrc/engine.hip

oracle:
	$(MAKE) -C oracle all

ref:
	$(MAKE) -C oracle ref

clean:
	rm -f kb2e_amd/libkb2e.so bin/kb2e $(BINS)
	$(MAKE) -C oracle clean

.PHONY: all oracle ref clean prof
