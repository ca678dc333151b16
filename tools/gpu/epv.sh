# Grouped epilogue variants (PR_EPI_VAR): GPU suite, s26 bench per variant, kernel trace of the default.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/epv
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/epv/pytest.log 2>&1 || exit 1
for V in 0 1 2 3 4; do
  PR_EPI_VAR=$V timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/epv/s26_v$V.log 2>&1 || exit 1
done
for V in 0 2; do
  PR_EPI_VAR=$V timeout -k 10 200 python -u bench.py --graph lj --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/epv/lj_v$V.log 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/epv/trace -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/epv/trace.log 2>&1
