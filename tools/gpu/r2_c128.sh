# Round 2: 128 column classes (four mask words per row) -- GPU tests of the class schedules, then
# A/B of the bench line at 64 vs 128 classes on s26, Twitter-shaped and ER s24 (kernel split by rocprofv3).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r2_c128; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 && \
for C in 64 128; do
  PR_CLASSES=$C timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/bench_s26_c$C.log 2>&1 || exit 1
  PR_CLASSES=$C timeout -k 10 200 python -u bench.py --no-cpu-baseline --graph twitter > $O/bench_tw_c$C.log 2>&1 || exit 1
  PR_CLASSES=$C timeout -k 10 200 python -u bench.py --no-cpu-baseline --graph er --scale 24 > $O/bench_er_c$C.log 2>&1 || exit 1
  PR_CLASSES=$C timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_c$C -o run -- python -u bench.py --no-cpu-baseline --steps 10 > $O/prof_c$C.log 2>&1 || exit 1
done
