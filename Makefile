# libspis.so — MI355X (gfx950) build of the CGMRES/FGMRES inner loop.  hipcc cross-compiles
# here (no GPU needed); the .so travels to the GPU box with the repo snapshot.
ROCM     ?= /opt/rocm
HIPCC    ?= $(ROCM)/bin/hipcc
ARCH     ?= gfx950
PKG      := structurepreservingiterativesolvers_amd
SRC      := $(PKG)/csrc
LIB      := $(PKG)/libspis.so
CXXFLAGS := -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -I include -I $(SRC)
HIPFLAGS := --offload-arch=$(ARCH) -munsafe-fp-atomics
OBJS     := build/kernels.o build/sptrsv.o build/spis.o build/lsq.o build/ilu_plan.o build/hash.o

all: $(LIB) $(PKG)/liblsq_host.so

build/kernels.o: $(SRC)/kernels.hip $(SRC)/kernels.h
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) $(CXXFLAGS) -c $< -o $@

build/spis.o: $(SRC)/spis.cpp $(SRC)/kernels.h $(SRC)/slab_order.h $(SRC)/col16.h $(SRC)/sptrsv.h $(SRC)/ilu_plan.h $(SRC)/lsq.h include/spis.h
	@mkdir -p build
	$(HIPCC) $(CXXFLAGS) -x hip --offload-arch=$(ARCH) -c $< -o $@

build/sptrsv.o: $(SRC)/sptrsv.hip $(SRC)/sptrsv.h $(SRC)/ilu_plan.h
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) $(CXXFLAGS) -c $< -o $@

build/ilu_plan.o: $(SRC)/ilu_plan.cpp $(SRC)/ilu_plan.h
	@mkdir -p build
	g++ $(CXXFLAGS) -c $< -o $@

build/hash.o: $(SRC)/hash.cpp include/spis.h
	@mkdir -p build
	g++ $(CXXFLAGS) -c $< -o $@

# the host least squares on x86-64-v3 (AVX2, FMA) with contraction off: the loops vectorise, every
# product is rounded then added as written, so results are bitwise the baseline build's
LSQFLAGS ?= -march=x86-64-v3 -ffp-contract=off

build/lsq.o: $(SRC)/lsq.cpp $(SRC)/lsq.h include/spis.h
	@mkdir -p build
	g++ $(CXXFLAGS) $(LSQFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $(OBJS) -L$(ROCM)/lib -lrccl -lpthread -Wl,-rpath,$(ROCM)/lib

# host-only build of the small dense LS for CPU unit tests (no HIP runtime needed)
$(PKG)/liblsq_host.so: $(SRC)/lsq.cpp $(SRC)/lsq.h $(SRC)/lsq_capi.cpp $(SRC)/ilu_plan.cpp $(SRC)/ilu_plan.h $(SRC)/ilu_capi.cpp \
                       $(SRC)/slab_order.h $(SRC)/col16.h $(SRC)/slab_capi.cpp
	g++ $(CXXFLAGS) $(LSQFLAGS) -shared -o $@ $(SRC)/lsq.cpp $(SRC)/lsq_capi.cpp $(SRC)/ilu_plan.cpp $(SRC)/ilu_capi.cpp $(SRC)/slab_capi.cpp

clean:
	rm -rf build $(LIB) $(PKG)/liblsq_host.so

.PHONY: all clean

# tuning tools (not built by default)
tools/chainbench: tools/chainbench.hip $(SRC)/kernels.hip $(SRC)/kernels.h
	$(HIPCC) $(HIPFLAGS) $(CXXFLAGS) -o $@ $<
tools/kbench: tools/kbench.hip $(SRC)/kernels.hip $(SRC)/kernels.h $(SRC)/slab_order.h $(SRC)/col16.h
	$(HIPCC) $(HIPFLAGS) $(CXXFLAGS) -o $@ $<

# tools/host_phases.py: spis_solve with its host phase marks compiled in (not the product library)
tools/libspis_phases.so: $(SRC)/spis.cpp $(OBJS)
	$(HIPCC) $(CXXFLAGS) -DSPIS_HOST_PHASES -x hip --offload-arch=$(ARCH) -c $< -o build/spis_phases.o
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $(filter-out build/spis.o,$(OBJS)) build/spis_phases.o -L$(ROCM)/lib -lrccl -lpthread -Wl,-rpath,$(ROCM)/lib

phases: tools/libspis_phases.so
