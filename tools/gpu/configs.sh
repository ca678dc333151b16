# Every BASELINE.json config through bench.py on the current default build (1 GPU).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/configs; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 150 python -u bench.py --scale 20 --steps 50 --warmup 5 --no-cpu-baseline > $O/rmat_s20.log 2>&1 && \
timeout -k 10 150 python -u bench.py --graph lj --steps 50 --warmup 5 --no-cpu-baseline > $O/lj.log 2>&1 && \
timeout -k 10 200 python -u bench.py --graph er --scale 24 --steps 20 --warmup 3 --no-cpu-baseline > $O/er_s24.log 2>&1 && \
timeout -k 10 300 python -u bench.py --graph twitter --steps 10 --warmup 2 --no-cpu-baseline > $O/twitter.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/rmat_s26.log 2>&1
