# HBM ceilings, then A/B bench of libmagent_cur vs libmagent_nt (nontemporal obs stores)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 120 python scripts/hbm_ceiling.py > gpurun_out/hbm_ceiling.json 2> gpurun_out/hbm_ceiling.err || exit 1
bash scripts/gpu_variants.sh cur nt cur nt
