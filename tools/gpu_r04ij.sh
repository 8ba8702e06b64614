# Round-4 GPU calls I + J in one: the octant chunk pipeline A/B (tools/gpu_r04i.sh), then the
# cell-wave C5 kernels (tools/gpu_r04j.sh).
set -e
cd $GRAFT_REPO_ROOT
bash tools/gpu_r04i.sh
cd $GRAFT_REPO_ROOT
bash tools/gpu_r04j.sh
