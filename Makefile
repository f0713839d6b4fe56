# Builds libsa_hip.so (the C-ABI hot-path library) for MI355X / gfx950.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH  ?= gfx950
SRC   := $(wildcard stereoanywhere_amd/csrc/*.hip)
HDR   := $(wildcard stereoanywhere_amd/csrc/*.h) include/stereoanywhere_hip.h
OUT   := stereoanywhere_amd/lib/libsa_hip.so
OBJ   := $(patsubst stereoanywhere_amd/csrc/%.hip,build/%.o,$(SRC))
# -ffp-contract=off: keep the reference's separate fp32 multiplies and adds
# (no fused multiply-add contraction) in the elementwise epilogues.
FLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-result

all: $(OUT)

# packed-f32 SLP vectorisation of the transform math costs register moves and spills beside
# the 144 MFMA accumulators (and packed VALU is no faster next to MFMAs).  Required, not a tuning
# knob: built without it the split instances spill 72-96 B per lane and failed the GPU tests (round
# 6); tests/test_kernel_resources.py checks this line and the no-spill build.
build/conv2d_wino4.o: FLAGS += -fno-slp-vectorize
# LLVM's wave-priority pass (s_setprio raised until a wave's first memory loads are issued, then
# lowered): conv2d_wino4 48.36 -> 47.42 ms/step, three interleaved passes (profiles/ab/r06_w4_wave_priority.txt)
build/conv2d_wino4.o: FLAGS += -mllvm -amdgpu-set-wave-priority

build/%.o: stereoanywhere_amd/csrc/%.hip $(HDR)
	@mkdir -p build
	$(HIPCC) $(FLAGS) -c $< -o $@

$(OUT): $(OBJ)
	@mkdir -p $(dir $@)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJ)

clean:
	rm -rf build $(OUT)

.PHONY: all clean
