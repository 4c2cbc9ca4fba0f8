# Round 5: 256x256 batch-size curve at S = 20 (2048 / 2560 / 3072 / 4096 envs): where the per-step time turns superlinear.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05r}
mkdir -p $O
for E in 2560 3072 4096 1536; do
timeout -k 10 300 python bench.py --map 256 --agents 4096 --envs $E --substeps 20 --steps 60 --warmup 10 --check-envs 2 --no-cpu-baseline > $O/e$E.json 2> $O/s.err || { tail -20 $O/s.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/e$E.json')); r=d['roofline']; print('E=$E %.4e frac %.4f ms/step %.4f kernel_ms %.3f check %s' % (d['value'], r['frac'], d['ms_per_step'], r.get('kernel_ms', -1), d.get('check', {}).get('ok')))"
done
