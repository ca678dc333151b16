set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/r9_pytest.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r9_bench26.log 2>&1
