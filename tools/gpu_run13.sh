set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=v4 STEPS=10 bash tools/profile.sh && \
timeout -k 10 300 python -u tools/diag_spmv.py --scale 26 --layout split --variants 0,1:6,1:12,1:19 > gpurun_out/r13_diag26.log 2>&1
