set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/diag_spmv.py --scale 26 --variants 0,7,8,9,4:19,10:19,11:19,4:22,10:22,11:22 > gpurun_out/r5_diag26.log 2>&1
