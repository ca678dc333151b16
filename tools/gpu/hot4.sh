# k_spmv_hot (DPP scan, lane metadata, 3-unit ring): parity, bench, diagnostic variants.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-hot4}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_bench.log 2>&1 && \
timeout -k 10 200 python -u tools/diag_spmv.py --scale 26 --layout split --variants ${VARS:-0,1,2,3} --rounds 3 --iters 5 > gpurun_out/${T}_diag.log 2>&1
