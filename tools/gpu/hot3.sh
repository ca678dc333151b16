# k_spmv_hot: parity at PT 8 and 16, then depth / store-flavour A/B at PT 8 and 16.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-hot3}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest8.log 2>&1 && \
PR_WAVE_PT=16 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k split > gpurun_out/${T}_pytest16.log 2>&1 && \
for PT in 8 16; do PR_WAVE_PT=$PT timeout -k 10 200 python -u tools/diag_spmv.py --scale 26 --layout split --variants ${VARS:-10,20,30,13,23,21,22} --rounds 3 --iters 5 > gpurun_out/${T}_diag_pt$PT.log 2>&1 || exit 1; done
