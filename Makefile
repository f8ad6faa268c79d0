# Build of the MI355X engine (in-tree, so the .so files travel to the GPU box).
#
#   make            -> zfec_amd/libzfec_hip.so  (C-ABI + HIP kernels, gfx950)
#                      zfec_amd/_fec<EXT>       (CPython extension, links the above)
#                      oracle/liboracle.so      (test-only CPU checker)
#   make ref        -> oracle/_ref/             (real reference, only where /root/reference exists)

HIPCC    ?= /opt/rocm/bin/hipcc
CXX      ?= g++
PY       ?= python3
ARCH     ?= gfx950
PYINC    := $(shell $(PY) -c "import sysconfig;print(sysconfig.get_paths()['include'])")
EXT      := $(shell $(PY) -c "import sysconfig;print(sysconfig.get_config_var('EXT_SUFFIX'))")
SRC      := zfec_amd/csrc
LIB      := zfec_amd/libzfec_hip.so
PYEXT    := zfec_amd/_fec$(EXT)
# every object depends on every header: config.hpp embeds bitslice.hpp's options, so a
# header change must rebuild all of them (a stale object reads a stale Config layout)
HDRS     := $(wildcard $(SRC)/*.hpp) $(SRC)/gf_routines.inc include/zfec_hip.h
HIPFLAGS := --offload-arch=$(ARCH) -mcode-object-version=5 -O3 -std=c++17 -fPIC -fvisibility=hidden -Wall -Wno-unused-function

all: $(LIB) $(PYEXT) oracle

$(SRC)/kernels.o: $(SRC)/kernels.hip $(HDRS)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(SRC)/bitslice.o: $(SRC)/bitslice.cpp $(HDRS)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(SRC)/fec_abi.o: $(SRC)/fec_abi.cpp $(HDRS)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(SRC)/gf256.o: $(SRC)/gf256.cpp $(HDRS)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(SRC)/host_pool.o: $(SRC)/host_pool.cpp $(HDRS)
	$(CXX) -O2 -std=c++17 -fPIC -fvisibility=hidden -Wall -c $< -o $@

$(SRC)/config.o: $(SRC)/config.cpp $(HDRS)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(SRC)/kernels.o $(SRC)/fec_abi.o $(SRC)/gf256.o $(SRC)/bitslice.o $(SRC)/host_pool.o $(SRC)/config.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -ldl -lpthread

$(PYEXT): $(SRC)/fecmodule.cpp include/zfec_hip.h $(LIB)
	$(CXX) -O2 -std=c++17 -fPIC -shared -fvisibility=hidden -I$(PYINC) -o $@ $< -Lzfec_amd -lzfec_hip -Wl,-rpath,'$$ORIGIN'

oracle:
	$(MAKE) -C oracle liboracle.so

# Host-code sanitizer builds (no GPU needed): every host object of the library
# compiled with AddressSanitizer / ThreadSanitizer (device code unchanged) and
# linked into tests/c/sanitize_driver.cpp, which runs the library's host-side
# concurrency and validation paths; the log goes to profiles/.
SANSRC   := $(SRC)/kernels.hip $(SRC)/fec_abi.cpp $(SRC)/gf256.cpp $(SRC)/bitslice.cpp $(SRC)/host_pool.cpp \
            $(SRC)/config.cpp tests/c/sanitize_driver.cpp
SANFLAGS := --offload-arch=$(ARCH) -mcode-object-version=5 -fPIC -O1 -g -fno-omit-frame-pointer -std=c++17 -Wall \
            -Wno-unused-function

build/%/driver: $(SANSRC) $(SRC)/*.hpp include/zfec_hip.h
	mkdir -p build/$*
	set -e; for f in $(SANSRC); do \
	  $(HIPCC) $(SANFLAGS) -Xarch_host -fsanitize=$* -c $$f -o build/$*/$$(basename $$f).o; done
	$(HIPCC) --offload-arch=$(ARCH) -fsanitize=$* -fno-gpu-sanitize -o $@ build/$*/*.o -ldl -lpthread

asan: build/address/driver
	ASAN_OPTIONS=detect_leaks=0 ./build/address/driver

tsan: build/thread/driver
	TSAN_OPTIONS="halt_on_error=0 second_deadlock_stack=1" ./build/thread/driver

# The no-GPU Python tests of the C-ABI (tests/test_cpu_surface.py: validation,
# JIT registry from threads) against an AddressSanitizer build of the library,
# loaded through zfec_amd.capi (ZFEC_HIP_LIB) with the ASan runtime preloaded.
ASANRT := $(shell $(HIPCC) -print-file-name=libclang_rt.asan-x86_64.so 2>/dev/null)
build/address/libzfec_hip.so: build/address/driver
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -fsanitize=address -shared-libasan -fno-gpu-sanitize -o $@ \
	  $(filter-out build/address/sanitize_driver.cpp.o,$(wildcard build/address/*.o)) -ldl -lpthread

asan-py: build/address/libzfec_hip.so
	ASAN_OPTIONS=detect_leaks=0 LD_PRELOAD=$(ASANRT) ZFEC_HIP_LIB=$(CURDIR)/build/address/libzfec_hip.so \
	  $(PY) -m pytest tests/test_cpu_surface.py -q -p no:cacheprovider \
	  -k "rejects or jit_prepare or fec_new or symbols or decode_matrix or invert_vdm or enc_matrix or batch_jobs"

ref:
	$(MAKE) -C oracle ref

clean:
	rm -f $(SRC)/*.o $(LIB) $(PYEXT)
	$(MAKE) -C oracle clean

.PHONY: all oracle ref clean asan tsan asan-py
