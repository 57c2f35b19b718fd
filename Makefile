# Build libocrk.so: every HIP kernel + the C-ABI, compiled for gfx950 only.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH  ?= gfx950
CSRC  := cnn_lstm_ctc_ocr_amd/csrc
HIPFLAGS := -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Iinclude -I$(CSRC) -Wall -Wno-unused-function
SRC   := $(wildcard $(CSRC)/*.hip)
OBJ   := $(patsubst $(CSRC)/%.hip,build/%.o,$(SRC))
HDR   := $(wildcard $(CSRC)/*.h) $(filter-out include/ocrk_comm.h,$(wildcard include/*.h))
LIB   := cnn_lstm_ctc_ocr_amd/libocrk.so
# the optional RCCL gradient all-reduce (include/ocrk_comm.h): its own object, so
# libocrk.so does not link RCCL
COMMLIB := cnn_lstm_ctc_ocr_amd/libocrk_comm.so

# built only where RCCL's header is present: libocrk.so never depends on it
RCCL_H := $(firstword $(wildcard /opt/rocm/include/rccl/rccl.h /opt/rocm/include/rccl.h))
ifeq ($(RCCL_H),)
all: $(LIB)
	@echo "rccl.h not found: $(COMMLIB) (optional all-reduce C ABI) not built"
else
all: $(LIB) $(COMMLIB)
endif

comm: $(COMMLIB)

$(COMMLIB): $(CSRC)/ocrk_comm.cpp include/ocrk_comm.h
	$(HIPCC) -O2 -std=c++17 -fPIC -shared -Iinclude -Wall -o $@ $< -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

$(LIB): $(OBJ)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $(OBJ)

build/%.o: $(CSRC)/%.hip $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# tools-only build: experiment toggles + diagnostics (include/ocrk_debug.h);
# tools load it with OCRK_LIB=tools/libocrk_exp.so. Never the product library.
EXPOBJ := $(patsubst $(CSRC)/%.hip,build/exp/%.o,$(SRC))
EXPLIB := tools/libocrk_exp.so

exp: $(EXPLIB)

$(EXPLIB): $(EXPOBJ)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $(EXPOBJ)

build/exp/%.o: $(CSRC)/%.hip $(HDR)
	@mkdir -p build/exp
	$(HIPCC) $(HIPFLAGS) -DOCRK_EXPERIMENTS -c $< -o $@

clean:
	rm -rf build $(LIB) $(COMMLIB) $(EXPLIB)

.PHONY: all comm exp clean
