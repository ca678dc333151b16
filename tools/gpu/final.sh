# Re-entry confirmation pass on the committed tree: GPU parity suite, smoke(), the default bench line
# (with the CPU baseline leg), and a rocprofv3 kernel trace of the same bench command.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/final; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/trace.log 2>&1
