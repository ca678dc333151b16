# 64 column classes: GPU suite, s26 at 32 / 64 classes, Twitter-shaped and LJ at 64, kernel trace at 64.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/c64
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/c64/pytest.log 2>&1 || exit 1
for C in 64 32; do
  PR_CLASSES=$C timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/c64/s26_c$C.log 2>&1 || exit 1
done
PR_CLASSES=64 timeout -k 10 300 python -u bench.py --graph twitter --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/c64/tw_c64.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --graph twitter --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/c64/tw_c32.log 2>&1 || exit 1
PR_CLASSES=64 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c64/trace -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/c64/trace.log 2>&1
