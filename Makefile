# Build everything in-tree (the built .so files travel to the GPU box with the
# repo snapshot; they are git-ignored).
#   make            libkb2e.so (HIP engine, gfx950) + oracle/liborc.so
#   make ref        also the reference build + fixture harness (needs /root/reference)
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS := --offload-arch=$(ARCH) -O3 -fPIC -std=c++17 -ffp-contract=off -Wall -Iinclude

CSRC := $(wildcard kb2e_amd/csrc/*.hip kb2e_amd/csrc/*.hpp kb2e_amd/csrc/*.inc) include/kb2e_engine.h

all: kb2e_amd/libkb2e.so oracle

kb2e_amd/libkb2e.so: $(CSRC)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ kb2e_amd/csrc/engine.hip

oracle:
	$(MAKE) -C oracle all

ref:
	$(MAKE) -C oracle ref

clean:
	rm -f kb2e_amd/libkb2e.so
	$(MAKE) -C oracle clean

.PHONY: all oracle ref clean
