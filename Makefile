# Builds the product library (HIP, gfx950) and the test-only CPU oracle.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CSRC := vectorscan_amd/csrc
LIB := vectorscan_amd/libvectorscan_amd.so
ORACLE := oracle/_build/liboracle.so
HARNESS := tests/c/abi_harness
HSNAMES := tests/c/hs_names_demo
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-function \
            -Wno-unused-parameter -Iinclude

DROPIN := tools/dropin_threads

all: $(LIB) $(ORACLE) $(HARNESS) $(HSNAMES) $(DROPIN)

$(CSRC)/compile.o: $(CSRC)/compile.cpp $(CSRC)/hs_layout.h $(CSRC)/vsa_internal.h
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(CSRC)/flood.o: $(CSRC)/flood.cpp $(CSRC)/hs_layout.h $(CSRC)/vsa_internal.h
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(CSRC)/hs_lit.o: $(CSRC)/hs_lit.cpp $(CSRC)/hs_layout.h $(CSRC)/vsa_internal.h \
                  include/vectorscan_amd.h include/vectorscan_amd_hs.h
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(CSRC)/kernels.o: $(CSRC)/kernels.hip $(CSRC)/kernels.h
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

RT_DEPS := $(CSRC)/runtime_internal.h $(CSRC)/kernels.h $(CSRC)/hs_layout.h \
           $(CSRC)/vsa_internal.h include/vectorscan_amd.h

# the host runtime: core, launch plans, drop-ins, batcher (runtime_internal.h)
$(CSRC)/runtime.o: $(CSRC)/runtime.hip $(RT_DEPS)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(CSRC)/plan.o: $(CSRC)/plan.hip $(RT_DEPS)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(CSRC)/dropin.o: $(CSRC)/dropin.hip $(RT_DEPS)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(CSRC)/batcher.o: $(CSRC)/batcher.hip $(RT_DEPS)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

RT_OBJS := $(CSRC)/runtime.o $(CSRC)/plan.o $(CSRC)/dropin.o $(CSRC)/batcher.o

$(LIB): $(CSRC)/compile.o $(CSRC)/flood.o $(CSRC)/hs_lit.o $(CSRC)/kernels.o $(RT_OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $^ -o $@

$(ORACLE): oracle/oracle.c
	mkdir -p oracle/_build
	gcc -O2 -march=x86-64-v3 -std=gnu11 -fPIC -shared -Wall -pthread $< -o $@

# test-only C caller of the drop-ins (real __m128i signatures), checked
# against the oracle
$(HARNESS): tests/c/abi_harness.c include/vectorscan_amd.h $(LIB) $(ORACLE)
	gcc -O2 -std=gnu11 -Wall -Iinclude $< -o $@ -Lvectorscan_amd -lvectorscan_amd \
	    -Loracle/_build -loracle -Wl,-rpath,'$$ORIGIN/../../vectorscan_amd' \
	    -Wl,-rpath,'$$ORIGIN/../../oracle/_build'

# test-only program written against the reference's hs names
# (include/vectorscan_amd_hs_names.h), checked against its own brute force
$(HSNAMES): tests/c/hs_names_demo.c include/vectorscan_amd_hs_names.h include/vectorscan_amd_hs.h $(LIB)
	gcc -O2 -std=gnu11 -Wall -Iinclude $< -o $@ -Lvectorscan_amd -lvectorscan_amd \
	    -Wl,-rpath,'$$ORIGIN/../../vectorscan_amd'

# measurement tool: small drop-in calls from POSIX threads (GPU, batcher,
# the oracle's SSE2 port as the CPU comparator)
$(DROPIN): tools/dropin_threads.c include/vectorscan_amd.h $(LIB) $(ORACLE)
	gcc -O2 -std=gnu11 -Wall -Iinclude $< -o $@ -Lvectorscan_amd -lvectorscan_amd \
	    -Loracle/_build -loracle -pthread -Wl,-rpath,'$$ORIGIN/../vectorscan_amd' \
	    -Wl,-rpath,'$$ORIGIN/../oracle/_build'

clean:
	rm -f $(CSRC)/*.o $(LIB) $(ORACLE) $(HARNESS) $(HSNAMES) $(DROPIN)

.PHONY: all clean
