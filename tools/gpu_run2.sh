set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/r2_pytest.log 2>&1 && \
timeout -k 10 300 python -u tools/diag_spmv.py --scale 26 > gpurun_out/r2_diag26.log 2>&1 && \
timeout -k 10 300 python -u tools/diag_spmv.py --scale 24 --graph er > gpurun_out/r2_diag_er24.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/r2_bench26.log 2>&1
