# Build a library variant for A/B benches: scripts/build_variant.sh NAME KERNEL_SOURCE [extra hipcc flags...]
# -> mean-field-multi-agent-reinforcement-learning_amd/build/libmagent_NAME.so (same flags as the Makefile)
set -e
P=/root/repo/mean-field-multi-agent-reinforcement-learning_amd
name=$1; src=$2; shift 2
cp "$src" $P/csrc/_variant_$name.hip
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fvisibility=hidden \
  -mllvm -amdgpu-atomic-optimizer-strategy=None "$@" -shared -Wl,-Bsymbolic -x hip $P/csrc/_variant_$name.hip \
  $P/csrc/battle_engine.cpp $P/csrc/mfx_common.cpp $P/csrc/ising_kernels.hip $P/csrc/ising_engine.cpp \
  $P/csrc/mf_kernels.hip $P/csrc/diag_kernels.hip $P/csrc/policy_kernels.hip $P/csrc/replay_kernels.hip \
  -o $P/build/libmagent_$name.so
rm -f $P/csrc/_variant_$name.hip
