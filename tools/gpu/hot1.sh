# Hot-set kernel: parity tests, bench line, hot-set size A/B (diagnostics library).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-hot1}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_bench.log 2>&1 && \
for K in 0 8192 18432; do PR_HOT_SLOTS=$K timeout -k 10 200 python -u tools/diag_spmv.py --scale 26 --layout split --variants 0 --rounds 3 --iters 5 > gpurun_out/${T}_diag_k$K.log 2>&1 || exit 1; done
