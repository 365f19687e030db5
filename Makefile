# Build of libsimilarity_transform.so (gfx950) and the CPU oracle.
# Usage: make [-j16]      (the same recipe __graft_entry__.build() runs)
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
# -fvisibility=hidden: the dynamic ABI is exactly what include/*.h declares
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off \
            -fno-fast-math -fvisibility=hidden -fvisibility-inlines-hidden \
            -Wall -Wextra -Wno-unused-parameter -Iinclude -Ieigen_value_amd/csrc
SRC      := eigen_value_amd/csrc/st_kernels.hip eigen_value_amd/csrc/st_solve.hip \
            eigen_value_amd/csrc/st_multi.hip eigen_value_amd/csrc/st_rendezvous.hip
OBJ      := $(patsubst eigen_value_amd/csrc/%.hip,build/%.o,$(SRC))
LIB      := eigen_value_amd/lib/libsimilarity_transform.so
# the tuning build (tools and the knob tests only): the same objects, with
# st_kernels compiled to also export the launch-table setters of
# include/st_tuning.h
TUNING_OBJ := build/st_kernels_tuning.o $(filter-out build/st_kernels.o,$(OBJ))
LIB_TUNING := eigen_value_amd/lib/libsimilarity_transform_tuning.so
HDRS     := include/similarity_transform.h include/st_tuning.h eigen_value_amd/csrc/st_internal.h \
            eigen_value_amd/csrc/st_device.h eigen_value_amd/csrc/st_rendezvous.h

all: $(LIB) $(LIB_TUNING) oracle

build/%.o: eigen_value_amd/csrc/%.hip $(HDRS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

build/st_kernels_tuning.o: eigen_value_amd/csrc/st_kernels.hip $(HDRS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -DST_TUNING_ABI=1 -c $< -o $@

$(LIB): $(OBJ)
	@mkdir -p eigen_value_amd/lib
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJ) -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

$(LIB_TUNING): $(TUNING_OBJ)
	@mkdir -p eigen_value_amd/lib
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(TUNING_OBJ) -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

# an A/B probe build of the launch-shape / kernel-code switches
# (st_kernels.hip, st_device.h): make probe PROBE="-DST_FLAT_ALT=0"; run a
# tool with EIGEN_VALUE_LIB pointing at the result (st_version names the
# switches); never a product build
PROBE_LIB := eigen_value_amd/lib/variants/libsimilarity_transform_probe.so
probe: $(SRC) $(HDRS)
	@mkdir -p build/probe eigen_value_amd/lib/variants
	for f in $(SRC); do $(HIPCC) $(HIPFLAGS) -DST_TUNING_ABI=1 -DST_PROBES=1 $(PROBE) \
	  -c $$f -o build/probe/$$(basename $$f .hip).o || exit 1; done
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $(PROBE_LIB) build/probe/*.o \
	  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf build eigen_value_amd/lib
	$(MAKE) -C oracle clean

.PHONY: all oracle clean probe
