set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/diag_spmv.py --scale 26 --variants 0,14,15,12 > gpurun_out/r6_diag26.log 2>&1 && \
timeout -k 10 300 python -u tools/diag_spmv.py --scale 24 --graph er --variants 0,14,15,12 > gpurun_out/r6_diag_er24.log 2>&1
