set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/diag_spmv.py --scale 26 --variants 0,4:6,4:9,4:12,4:15,4:17,4:19,5:12,6:12,5:19,6:19 > gpurun_out/r3_diag26.log 2>&1
