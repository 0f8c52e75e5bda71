# Builds libdwpa22000.so (HIP for gfx950 + host C++) in-tree, and the CPU parity oracle (test infrastructure).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CXXFLAGS ?= -O3 -std=c++17 -fPIC -Wall -Wno-unused-function
SRC := dwpa_amd/csrc
OBJ := build/obj
LIB := dwpa_amd/lib/libdwpa22000.so
HDRS := $(wildcard $(SRC)/*.hpp) include/dwpa22000.h
OBJS := $(OBJ)/kernels.o $(OBJ)/rules_dev.o $(OBJ)/engine.o $(OBJ)/m22000_host.o $(OBJ)/crack.o $(OBJ)/rules.o \
        $(OBJ)/pbkdf2_module.o $(OBJ)/pbkdf2_hsaco.o $(OBJ)/host_crypto.o $(OBJ)/host_check.o
LLVM := /opt/rocm/lib/llvm/bin
ISSUE_RULE ?= sched=1:alt:orig:asmnop,before_half

all: $(LIB) oracle

$(OBJ)/%.o: $(SRC)/%.hip $(HDRS)
	@mkdir -p $(OBJ)
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) -Iinclude -c $< -o $@

$(OBJ)/%.o: $(SRC)/%.cpp $(HDRS)
	@mkdir -p $(OBJ)
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) -Iinclude -c $< -o $@

# product PBKDF2 kernel: hipcc -> gfx950 asm -> VALU issue pass -> code object -> embedded byte array
build/pbkdf2/pbkdf2_gfx950.s: $(SRC)/pbkdf2_gfx950.hip $(SRC)/pbkdf2_dev.hpp $(SRC)/crypto_dev.hpp
	@mkdir -p build/pbkdf2
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 --cuda-device-only -S $< -o $@

PBKDF2_KERNELS := k_pbkdf2_gfx950+k_pbkdf2_gfx950_ms+k_pbkdf2_gfx950_mg+k_pbkdf2_gfx950_p+k_pbkdf2_gfx950_ms_p+k_pbkdf2_gfx950_mg_p+k_pbkdf2_gfx950_q+k_pbkdf2_gfx950_mg_q

# the pass fails closed (an instruction it cannot model stops the build) ...
build/pbkdf2/pbkdf2_issue.s: build/pbkdf2/pbkdf2_gfx950.s $(SRC)/gen/issue_pass.py Makefile
	python3 $(SRC)/gen/issue_pass.py $< $@ $(PBKDF2_KERNELS) $(ISSUE_RULE)

# ... and every scheduled loop must compute the compiler's results (tools/issue_equiv.py) before the code object links
build/pbkdf2/issue_equiv.ok: build/pbkdf2/pbkdf2_gfx950.s build/pbkdf2/pbkdf2_issue.s tools/issue_equiv.py
	python3 tools/issue_equiv.py $< $(PBKDF2_KERNELS) $(ISSUE_RULE) 2
	@touch $@

build/pbkdf2/pbkdf2_gfx950.hsaco: build/pbkdf2/pbkdf2_issue.s build/pbkdf2/issue_equiv.ok
	$(LLVM)/clang -target amdgcn-amd-amdhsa -mcpu=$(ARCH) -c $< -o build/pbkdf2/pbkdf2_issue.o
	$(LLVM)/ld.lld -shared build/pbkdf2/pbkdf2_issue.o -o $@

build/pbkdf2/pbkdf2_hsaco.cpp: build/pbkdf2/pbkdf2_gfx950.hsaco $(SRC)/gen/embed.py
	python3 $(SRC)/gen/embed.py $< $@ pbkdf2_gfx950_hsaco

$(OBJ)/pbkdf2_hsaco.o: build/pbkdf2/pbkdf2_hsaco.cpp
	@mkdir -p $(OBJ)
	$(HIPCC) $(CXXFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	@mkdir -p dwpa_amd/lib
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS) -lz -lpthread

oracle:
	$(MAKE) -s -C oracle

asm: $(SRC)/kernels.hip $(HDRS)
	@mkdir -p build/asm
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) -Iinclude -c $< -o build/asm/kernels.o -save-temps=obj -Rpass-analysis=kernel-resource-usage

clean:
	rm -rf build $(LIB)
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean asm

tools: tools/bin/valu_peak tools/bin/pbkdf2_lab tools/bin/valu_lat tools/bin/valu_peak64 tools/bin/inflate_bench \
       tools/bin/inflate_check tools/bin/item_queue_check tools/bin/rules_fuzz_asan tools/bin/clock_idle \
       tools/bin/inflate_check_tsan tools/bin/tail_placement tools/bin/parse_fuzz_asan tools/bin/host_check_fuzz_asan tools/bin/host_pbkdf2_paths tools/bin/vgpr_bank

tools/bin/valu_lat: tools/valu_lat.hip
	@mkdir -p tools/bin
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -o $@ $<

tools/bin/pbkdf2_lab: tools/pbkdf2_lab.hip dwpa_amd/csrc/crypto_dev.hpp
	@mkdir -p tools/bin
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -o $@ $<

tools/bin/valu_peak: tools/valu_peak.hip
	@mkdir -p tools/bin
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -o $@ $<

.PHONY: tools

tools/bin/valu_peak64: tools/valu_peak64.hip
	@mkdir -p tools/bin
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -o $@ $<

tools/bin/inflate_bench: tools/inflate_bench.cpp $(SRC)/dict_reader.hpp $(SRC)/inflate.hpp $(SRC)/pinflate.hpp $(SRC)/m22000_host.cpp \
                         $(SRC)/m22000_host.hpp
	@mkdir -p tools/bin
	g++ -O3 -std=c++17 -Iinclude -I$(SRC) -o $@ tools/inflate_bench.cpp $(SRC)/m22000_host.cpp -lz -lpthread

tools/bin/inflate_check: tools/inflate_check.cpp $(SRC)/inflate.hpp $(SRC)/pinflate.hpp
	@mkdir -p tools/bin
	g++ -O3 -std=c++17 -Wall -I$(SRC) -o $@ tools/inflate_check.cpp -lz -lpthread

tools/bin/item_queue_check: tools/item_queue_check.cpp $(SRC)/dict_reader.hpp $(SRC)/inflate.hpp $(SRC)/pinflate.hpp \
                            $(SRC)/m22000_host.cpp $(SRC)/m22000_host.hpp
	@mkdir -p tools/bin
	g++ -O2 -std=c++17 -Wall -Iinclude -I$(SRC) -o $@ tools/item_queue_check.cpp $(SRC)/m22000_host.cpp -lz -lpthread

# host fuzz of the rule engine under AddressSanitizer + UBSan (host code only: -fsanitize after -Xarch_host)
tools/bin/rules_fuzz_asan: tools/rules_fuzz.cpp $(SRC)/rules.cpp $(SRC)/rules.hpp $(SRC)/rules_apply.hpp
	@mkdir -p tools/bin
	$(HIPCC) -O1 -g -std=c++17 -Iinclude -I$(SRC) -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined \
	    -o $@ tools/rules_fuzz.cpp $(SRC)/rules.cpp

tools/bin/parse_fuzz_asan: tools/parse_fuzz.cpp $(SRC)/m22000_host.cpp $(SRC)/m22000_host.hpp $(SRC)/tables.hpp
	@mkdir -p tools/bin
	$(HIPCC) -O1 -g -std=c++17 -Iinclude -I$(SRC) -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined \
	    -o $@ tools/parse_fuzz.cpp $(SRC)/m22000_host.cpp

# host fuzz of the host backend's check path under AddressSanitizer + UBSan (the engine's thread pool stubbed)
tools/bin/host_check_fuzz_asan: tools/host_check_fuzz.cpp $(SRC)/host_check.cpp $(SRC)/host_crypto.cpp \
                                $(SRC)/host_crypto.hpp $(SRC)/m22000_host.cpp $(SRC)/m22000_host.hpp $(SRC)/engine.hpp
	@mkdir -p tools/bin
	$(HIPCC) -O1 -g -std=c++17 -Iinclude -I$(SRC) -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined \
	    -o $@ tools/host_check_fuzz.cpp $(SRC)/host_check.cpp $(SRC)/host_crypto.cpp $(SRC)/m22000_host.cpp -lpthread

# one thread's time per call of each host PBKDF2 loop (SHA-NI 1/2/4 chains, AVX-512 1/2/3 registers, scalar)
tools/bin/host_pbkdf2_paths: tools/host_pbkdf2_paths.cpp $(SRC)/host_crypto.cpp $(SRC)/host_crypto.hpp
	@mkdir -p tools/bin
	$(HIPCC) -O3 -std=c++17 -Iinclude -I$(SRC) -o $@ tools/host_pbkdf2_paths.cpp

tools/bin/clock_idle: tools/clock_idle.hip
	@mkdir -p tools/bin
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -o $@ $<

tools/bin/vgpr_bank: tools/vgpr_bank.hip
	@mkdir -p tools/bin
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -o $@ $<

tools/bin/tail_placement: tools/tail_placement.hip
	@mkdir -p tools/bin
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -o $@ $<

# the parallel inflate (loader thread + workers + the reader) under ThreadSanitizer
tools/bin/inflate_check_tsan: tools/inflate_check.cpp $(SRC)/inflate.hpp $(SRC)/pinflate.hpp
	@mkdir -p tools/bin
	g++ -O1 -g -std=c++17 -Wall -I$(SRC) -fsanitize=thread -DDWPA_PINFLATE_LOAD_STEP=16384 -o $@ tools/inflate_check.cpp \
	    -lz -lpthread
