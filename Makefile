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
HIPFLAGS := --offload-arch=$(ARCH) -mcode-object-version=5 -O3 -std=c++17 -fPIC -fvisibility=hidden -Wall -Wno-unused-function

all: $(LIB) $(PYEXT) oracle

$(SRC)/kernels.o: $(SRC)/kernels.hip $(SRC)/kernels.hpp $(SRC)/bitslice.hpp
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(SRC)/bitslice.o: $(SRC)/bitslice.cpp $(SRC)/bitslice.hpp $(SRC)/kernels.hpp $(SRC)/gf256.hpp
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(SRC)/fec_abi.o: $(SRC)/fec_abi.cpp $(SRC)/kernels.hpp $(SRC)/gf256.hpp $(SRC)/host_pool.hpp include/zfec_hip.h
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(SRC)/gf256.o: $(SRC)/gf256.cpp $(SRC)/gf256.hpp
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(SRC)/host_pool.o: $(SRC)/host_pool.cpp $(SRC)/host_pool.hpp
	$(CXX) -O2 -std=c++17 -fPIC -fvisibility=hidden -Wall -c $< -o $@

$(LIB): $(SRC)/kernels.o $(SRC)/fec_abi.o $(SRC)/gf256.o $(SRC)/bitslice.o $(SRC)/host_pool.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -ldl -lpthread

$(PYEXT): $(SRC)/fecmodule.cpp include/zfec_hip.h $(LIB)
	$(CXX) -O2 -std=c++17 -fPIC -shared -fvisibility=hidden -I$(PYINC) -o $@ $< -Lzfec_amd -lzfec_hip -Wl,-rpath,'$$ORIGIN'

oracle:
	$(MAKE) -C oracle liboracle.so

ref:
	$(MAKE) -C oracle ref

clean:
	rm -f $(SRC)/*.o $(LIB) $(PYEXT)
	$(MAKE) -C oracle clean

.PHONY: all oracle ref clean
