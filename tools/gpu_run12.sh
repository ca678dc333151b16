set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/diag_spmv.py --scale 26 --layout split --variants 0,1:6,1:12,1:19 > gpurun_out/r12_diag26.log 2>&1
