# Builds libbcmpc.so (HIP for gfx950) in-tree.  `make -j` is safe; no cmake.
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -ffp-contract=off -fno-slp-vectorize -Wall -Wno-unused-function
SRC      := bc_mpc_amd/csrc
LIB      := bc_mpc_amd/libbcmpc.so
OBJ      := build/rollout.o build/capi.o
HDR      := include/bcmpc.h $(SRC)/kernels.h

all: $(LIB)

build/rollout.o: $(SRC)/rollout.hip $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

build/capi.o: $(SRC)/capi.cpp $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(LIB): $(OBJ)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(OBJ)

# resource usage report (VGPR/SGPR/LDS/occupancy) for the rollout kernels
resources: $(SRC)/rollout.hip $(HDR)
	$(HIPCC) $(HIPFLAGS) -c $< -o /dev/null -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E "Function Name|VGPRs:|AGPRs|Spill|Occupancy|LDS" 

asm: $(SRC)/rollout.hip $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -S --cuda-device-only $< -o build/rollout.s

clean:
	rm -rf build $(LIB)

.PHONY: all clean resources asm
