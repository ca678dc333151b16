set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/r1_pytest.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r1_smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py --scale 22 --steps 10 --warmup 2 --cpu-budget-s 5 > gpurun_out/r1_bench22.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 > gpurun_out/r1_bench26.log 2>&1
