# Build the product library (librein48.so: gfx950 kernels + C-ABI) and the test-only oracle.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 --offload-arch=$(ARCH) -fPIC -Wall -Wno-unused-function
LIBDIR := rein48_amd/lib
SRC := rein48_amd/csrc/r48_env.hip rein48_amd/csrc/r48_a3c.hip rein48_amd/csrc/r48_policy.hip rein48_amd/csrc/r48_replay.hip rein48_amd/csrc/r48_dqn.hip rein48_amd/csrc/r48_resnet.hip rein48_amd/csrc/r48_a3c_train.hip rein48_amd/csrc/r48_bn.hip rein48_amd/csrc/r48_conv.hip rein48_amd/csrc/r48_game.hip rein48_amd/csrc/r48_mlp.hip rein48_amd/csrc/r48_mlp_train.hip
DEPS := rein48_amd/csrc/r48_host.h rein48_amd/csrc/r48_board.h rein48_amd/csrc/r48_cnn_common.h rein48_amd/csrc/r48_mlp_common.h rein48_amd/csrc/r48_bn_finish.h include/rein48.h

all: $(LIBDIR)/librein48.so oracle

OBJDIR := build/obj
OBJ := $(patsubst rein48_amd/csrc/%.hip,$(OBJDIR)/%.o,$(SRC))
# the fused A3C update keeps its loop-carried gradient slices in AGPRs and its MFMA results in
# VGPRs (no accumulator round trips through v_accvgpr_read before each epilogue); LLVM's
# max-memory-clause machine scheduler: -1.5 % per 10^8 rows, bit-identical (four alternated rounds,
# process per library, A/A control: profiles/r06/a3c/train/sched_strategy_ab.txt)
FLAGS_r48_a3c_train := -mllvm -amdgpu-mfma-vgpr-form=1 -mllvm -amdgpu-sched-strategy=max-memory-clause
# the CNN rollout megakernel: the max-ILP machine scheduler (rollout 7.82 -> 7.70 ms textbook, 7.46 -> 7.35 ms
# reference over 4 alternated samples each, profiles/r04/a3c/rollout_sched_max_ilp_ab.txt)
FLAGS_r48_policy ?= -mllvm -amdgpu-sched-strategy=max-ilp
# the cell-grouped ResNet kernel keeps its 16 x 4 live accumulators in VGPRs (the epilogue reads
# them without v_accvgpr_read) and the block input in AGPRs
FLAGS_r48_resnet ?= -mllvm -amdgpu-mfma-vgpr-form=1
# the MLP policy: its layer-1 f32 MFMA results stay in VGPRs for the VALU layer 2 (rollout 6.24 -> 5.90 ms
# reference, 3.49 -> 3.39 ms textbook vs the AGPR form, profiles/r05/a3c/mlp_policy_f32_mfma_ab.txt)
FLAGS_r48_mlp ?= -mllvm -amdgpu-mfma-vgpr-form=1
# the MLP update: no SLP packing of its scalar f32 adds / FMAs (packed f32 VALU issues at half rate)
FLAGS_r48_mlp_train ?= -fno-slp-vectorize

$(LIBDIR)/librein48.so: $(OBJ)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(OBJ)

$(OBJDIR)/%.o: rein48_amd/csrc/%.hip $(DEPS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) $(FLAGS_$*) -c -o $@ $<

# assembly + register report for the hot kernels (not needed for the build)
asm: $(SRC) $(DEPS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) --cuda-device-only -S -o build/r48_env.s rein48_amd/csrc/r48_env.hip
	$(HIPCC) $(HIPFLAGS) --cuda-device-only -S -o build/r48_a3c.s rein48_amd/csrc/r48_a3c.hip
	$(HIPCC) $(HIPFLAGS) --cuda-device-only -S -o build/r48_policy.s rein48_amd/csrc/r48_policy.hip
	$(HIPCC) $(HIPFLAGS) --cuda-device-only -c -o /dev/null -Rpass-analysis=kernel-resource-usage rein48_amd/csrc/r48_policy.hip 2> build/resource_usage_policy.txt
	$(HIPCC) $(HIPFLAGS) --cuda-device-only -c -o /dev/null -Rpass-analysis=kernel-resource-usage rein48_amd/csrc/r48_env.hip 2> build/resource_usage.txt

oracle:
	$(MAKE) -s -C oracle

clean:
	rm -rf $(LIBDIR) build
	$(MAKE) -s -C oracle clean

.PHONY: all asm oracle clean
