# 64 classes by default + leaner grouped epilogue: GPU suite, s26 (64 / 32 classes), Twitter, LJ, trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/c64b; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/s26.log 2>&1 || exit 1
PR_CLASSES=32 timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/s26_c32.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --graph twitter --steps 10 --warmup 2 --no-cpu-baseline > $O/tw.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --graph lj --steps 30 --warmup 3 --no-cpu-baseline > $O/lj.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/trace.log 2>&1
