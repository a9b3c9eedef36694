# Builds libbcmpc.so (HIP for gfx950) in-tree.  `make -j` is safe; no cmake.
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -ffp-contract=off -fno-slp-vectorize -Wall -Wno-unused-function
SRC      := bc_mpc_amd/csrc
LIB      := bc_mpc_amd/libbcmpc.so
OBJ      := build/rollout.o build/rollout_grp.o build/rollout_x3.o build/rollout_x3_plain.o build/rollout_team.o build/cem.o build/fit.o build/capi.o build/mt19937.o build/mt_jump.o build/mt_device.o build/comm.o
HDR      := include/bcmpc.h $(SRC)/kernels.h $(SRC)/device_common.h $(SRC)/argmin_common.h

all: $(LIB)

build/rollout.o: $(SRC)/rollout.hip $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

build/rollout_grp.o: $(SRC)/rollout_grp.hip $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# the split kernel in two units (X3_PART in rollout_x3.hip), each with the scheduler that measured best
# (profiles/r01_sched_ilp_ab.txt, profiles/r01_sched_part2_ab.txt): the plain tanh delta net with
# iterative-ILP (-1..2% kernel time at cfg3/cfg4), the policy / reward / relu-LN kernels with max-ILP
# (-0.6..1.7%; iterative-ILP spills the policy+reward kernel, +10%)
X3ILP    ?= -mllvm -amdgpu-sched-strategy=iterative-ilp
X3P2     ?= -mllvm -amdgpu-sched-strategy=max-ilp

build/rollout_x3.o: $(SRC)/rollout_x3.hip $(HDR) $(SRC)/split_common.h
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) $(X3P2) -DX3_PART=2 -c $< -o $@

build/rollout_x3_plain.o: $(SRC)/rollout_x3.hip $(HDR) $(SRC)/split_common.h
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) $(X3ILP) -DX3_PART=1 -c $< -o $@

# the team kernels with the iterative ILP scheduler: ppo_defaults -2.4 us, ppo_mpc_default -5.5 us, run.sh
# recipe -4.8 us per call against the default (max-ilp +2.5..+21 us, iterative-minreg +0..+24 us;
# profiles/r04_team_sched_ab.jsonl)
TEAMSCHED ?= -mllvm -amdgpu-sched-strategy=iterative-ilp
build/rollout_team.o: $(SRC)/rollout_team.hip $(HDR) $(SRC)/split_common.h
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) $(TEAMSCHED) -c $< -o $@

build/fit.o: $(SRC)/fit.hip $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

build/mt_device.o: $(SRC)/mt_device.hip $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

build/comm.o: $(SRC)/comm.hip $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

build/cem.o: $(SRC)/cem.hip $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

build/mt19937.o: $(SRC)/mt19937.cpp $(SRC)/mt19937.h
	@mkdir -p build
	g++ -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -c $< -o $@

build/mt_jump.o: $(SRC)/mt_jump.cpp $(SRC)/mt19937.h
	@mkdir -p build
	g++ -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -c $< -o $@

build/capi.o: $(SRC)/capi.cpp $(HDR) $(SRC)/mt19937.h
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(LIB): $(OBJ)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(OBJ) -ldl

# resource usage report (VGPR/SGPR/LDS/occupancy) for the rollout kernels
resources: $(SRC)/rollout.hip $(SRC)/rollout_grp.hip $(HDR)
	$(HIPCC) $(HIPFLAGS) -c $(SRC)/rollout.hip -o /dev/null -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E "Function Name|VGPRs:|AGPRs|Spill|Occupancy|LDS"
	$(HIPCC) $(HIPFLAGS) -c $(SRC)/rollout_grp.hip -o /dev/null -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E "Function Name|VGPRs:|AGPRs|Spill|Occupancy|LDS" 

asm: $(SRC)/rollout.hip $(SRC)/rollout_grp.hip $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -S --cuda-device-only $(SRC)/rollout.hip -o build/rollout.s
	$(HIPCC) $(HIPFLAGS) -S --cuda-device-only $(SRC)/rollout_grp.hip -o build/rollout_grp.s

clean:
	rm -rf build $(LIB)

.PHONY: all clean resources asm
