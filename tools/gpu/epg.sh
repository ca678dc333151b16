# Grouped epilogue (k_epilogue_grp): GPU suite, bench s26 A/B (PR_EPI_GRP, PR_EPI_WIN), LJ, kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/epg
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/epg/pytest.log 2>&1 || exit 1
for D in 2048 1024; do
  PR_EPI_WIN=$D timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/epg/s26_w$D.log 2>&1 || exit 1
done
PR_EPI_GRP=0 timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/epg/s26_g0.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --graph lj --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/epg/lj.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/epg/trace -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/epg/trace.log 2>&1 || exit 1
PR_EPI_WIN=1024 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/epg/trace1024 -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/epg/trace1024.log 2>&1
