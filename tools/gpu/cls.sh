# Column classes 8 / 16 / 32: parity at the non-default counts, then the iteration time.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-cls}
PR_CLASSES=32 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k split > gpurun_out/${T}_pytest32.log 2>&1 && \
PR_CLASSES=8 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k split > gpurun_out/${T}_pytest8.log 2>&1 && \
for C in ${CLS:-8 16 32}; do PR_CLASSES=$C timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 > gpurun_out/${T}_bench_c$C.log 2>&1 || exit 1; done
