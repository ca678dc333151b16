# A/B: per-XCD phased class schedule (PR_HOT_PHASED) x column classes, bench s26 + split parity.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ph
export TMPDIR=/tmp
PR_HOT_PHASED=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "split or rmat or lj" --timeout 120 --timeout-method thread > gpurun_out/ph/pytest.log 2>&1 || exit 1
PR_HOT_PHASED=1 PR_CLASSES=32 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "rmat or lj" --timeout 120 --timeout-method thread > gpurun_out/ph/pytest32.log 2>&1 || exit 1
for C in 16 32; do
  for PH in 0 1; do
    PR_HOT_PHASED=$PH PR_CLASSES=$C timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ph/bench_c${C}_p${PH}.log 2>&1 || exit 1
  done
done
