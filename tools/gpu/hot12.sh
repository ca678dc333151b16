# Full GPU parity suite, then the heavy-row kernel's issue-order A/B (diagnostics library).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-hot12}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && \
timeout -k 10 200 python -u tools/diag_spmv.py --scale 26 --layout split --variants ${VARS:-0,13,1,14,4,15} --rounds 3 --iters 5 > gpurun_out/${T}_diag.log 2>&1
