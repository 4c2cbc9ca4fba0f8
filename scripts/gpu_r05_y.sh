# Round 5: Ising stream mode at 16384 replicas: scan ring 24 / 32 blocks and the gen stream's priority (A/B).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05y}
mkdir -p $O
for C in "32 x" "24 x" "32 -1" "32 1" "24 -1" "32 x"; do
set -- $C; RB=$1; PR=$2
if [ $PR = x ]; then unset MFX_ISING_GEN_PRIO; else export MFX_ISING_GEN_PRIO=$PR; fi
MFX_ISING_SCAN_RING=$RB timeout -k 10 300 python scripts/bench_ising.py --mode reference --replicas 16384 --no-cpu > $O/b.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b.json')); print('ring=$RB prio=$PR value %.4e call %.4f' % (d['value'], d['seconds_call']))"
done
