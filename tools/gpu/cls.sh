# Column classes 8 vs 16 (x heavy threshold): parity at 16, then timing of the whole iteration.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-cls}
PR_CLASSES=16 PR_HEAVY_MIN=16 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest16.log 2>&1 && \
for CFG in "8 8" "16 16" "16 12" "16 24"; do set -- $CFG; PR_CLASSES=$1 PR_HEAVY_MIN=$2 timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 > gpurun_out/${T}_bench_c$1_h$2.log 2>&1 || exit 1; done
