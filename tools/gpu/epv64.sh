# Epilogue (group, window) variants at 64 column classes (R-MAT s26): PR_EPI_VAR 0..4.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/epv64; mkdir -p $O
export TMPDIR=/tmp
for v in 0 1 4 2 3; do
  PR_EPI_VAR=$v timeout -k 10 150 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/var$v.log 2>&1 || exit 1
done
