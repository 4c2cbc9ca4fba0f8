# Round 3: re-seed A/B + new tests + bench + GPU suite, then the configs[3] small-E sweep.
cd $GRAFT_REPO_ROOT
bash scripts/gpu_r03_reseed_ab.sh; rc=$?
echo "reseed_ab exit $rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash scripts/gpu_r03_small_e.sh
