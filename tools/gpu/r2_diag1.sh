# Round 2, first box: GPU tests on the current build + k_spmv_hot issue-cost diagnostics at s26.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r2_diag1; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 300 python -u tools/diag_spmv.py --scale 26 --layout split --variants 16,17,18,19 --rounds 3 --iters 5 > $O/diag_s26.log 2>&1 && \
timeout -k 10 300 python -u tools/diag_spmv.py --scale 24 --graph er --layout split --variants 16,17,18,19 --rounds 3 --iters 5 > $O/diag_er24.log 2>&1
