# Round 5: Ising stream mode at 16384 replicas: pass size (MFX_ISING_PASS_GB) x scan ring (A/B).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05z}
mkdir -p $O
for C in "16 24" "32 24" "64 24" "48 24" "16 32"; do
set -- $C; G=$1; RB=$2
MFX_ISING_PASS_GB=$G MFX_ISING_SCAN_RING=$RB timeout -k 10 300 python scripts/bench_ising.py --mode reference --replicas 16384 --no-cpu > $O/b.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b.json')); print('pass_gb=$G ring=$RB value %.4e call %.4f' % (d['value'], d['seconds_call']))"
done
