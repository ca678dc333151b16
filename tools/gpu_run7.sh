set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/r7_pytest.log 2>&1 && \
timeout -k 10 300 python -u tools/diag_spmv.py --scale 26 --variants 0,14,15,12 > gpurun_out/r7_diag26.log 2>&1 && \
TAG=v2 STEPS=10 bash tools/profile.sh
