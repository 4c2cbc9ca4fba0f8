# bench several library variants back to back: scripts/gpu_variants.sh name1 name2 ...
# -> gpurun_out/var_<name>_<k>.json (k = position in the argument list)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
B=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build
k=0
for n in "$@"; do
  k=$((k+1))
  MAGENT_LIB=$B/libmagent_$n.so timeout -k 10 300 python bench.py --steps 50 --warmup 5 --envs 16384 --no-cpu-baseline > gpurun_out/var_${n}_$k.json 2> gpurun_out/var_${n}_$k.err || exit 1
done
