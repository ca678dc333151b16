set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/diag_spmv.py --scale 26 --variants 0,16,17,18 > gpurun_out/r8_diag26.log 2>&1
