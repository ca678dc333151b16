# Split threshold at 4 MiB: GPU parity suite, smoke, R-MAT s20 (now split, 8 classes), LJ and s26 lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/thresh; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 150 python -u bench.py --scale 20 --steps 100 --warmup 10 > $O/rmat_s20.log 2>&1 && \
timeout -k 10 150 python -u bench.py --graph lj --steps 50 --warmup 5 --no-cpu-baseline > $O/lj.log 2>&1 && \
timeout -k 10 300 python -u bench.py > $O/rmat_s26.log 2>&1
