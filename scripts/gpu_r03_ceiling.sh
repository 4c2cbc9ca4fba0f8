# Round 3: k_rollout against the write ceilings of ONE box, interleaved after a warm-up bench: its own
# store pattern without compute (scripts/micro/write_pattern), torch fill / copy / sum
# (scripts/hbm_ceiling.py), and the default bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03ceil
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench0.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
for r in 1 2 3; do
timeout -k 10 120 ./scripts/micro/write_pattern > $O/write_pattern$r.txt 2>&1 || { cat $O/write_pattern$r.txt; exit 1; }
grep -E "regions +nt=1 wg/cu=5|fill" $O/write_pattern$r.txt
timeout -k 10 200 python scripts/hbm_ceiling.py > $O/hbm_ceiling$r.json 2> $O/hbm.err || { tail -5 $O/hbm.err; exit 1; }
cat $O/hbm_ceiling$r.json
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench$r.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench$r.json')); r=d['roofline']; print('bench %.4e frac %.4f achieved %.1f GB/s' % (d['value'], r['frac'], r['achieved']))"
done
