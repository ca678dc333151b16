# A/B: epilogue slot addressing (PR_EPI_ABS) - split parity, then bench s26 both ways + trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/epi
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "split or rmat or lj or group" --timeout 120 --timeout-method thread > gpurun_out/epi/pytest.log 2>&1 || exit 1
for D in 0 1; do
  PR_EPI_ABS=$D timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/epi/bench_a$D.log 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/epi/trace -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/epi/trace.log 2>&1
