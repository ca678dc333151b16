set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/diag_spmv.py --scale 26 --layout split --variants 0,2,3,4,0,2,4 > gpurun_out/r14_diag26.log 2>&1
