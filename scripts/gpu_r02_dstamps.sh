# Phase stamps of the resident drop-in server (diagnostic build) at 40x40: device phases and the
# host-side split of env.step(), for the poll / answer variants (MFX_DROPIN_VARIANT).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02s
mkdir -p $O
export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build/libmagent_stamps.so
for v in 0; do
  MFX_DROPIN_VARIANT=$v MAGENT_LIB=$L timeout -k 10 120 python scripts/stamps_dropin.py --map 40 --agents 128 > $O/stamps40_v$v.txt 2>&1 || { cat $O/stamps40_v$v.txt; exit 1; }
  echo "variant $v"; grep -h "map\|stamps" $O/stamps40_v$v.txt
done
