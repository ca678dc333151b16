# LJ-shaped: class count x phased schedule.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ljab
export TMPDIR=/tmp
for CP in 8:0 16:0 16:1 32:0 32:1; do
  C=${CP%:*}; P=${CP#*:}
  PR_CLASSES=$C PR_HOT_PHASED=$P timeout -k 10 200 python -u bench.py --graph lj --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/ljab/c${C}_p${P}.log 2>&1 || exit 1
done
