# R-MAT s20 (configs[0], 5 MB gather space): fused layout (auto) vs the split layout at 8 / 16 classes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/s20_ab; mkdir -p $O
export TMPDIR=/tmp
s20() { timeout -k 10 150 python -u bench.py --scale 20 --steps 100 --warmup 10 --no-cpu-baseline "${@:2}" > $O/s20_$1.log 2>&1; }
s20 auto && s20 split8 --layout split && PR_CLASSES=16 s20 split16 --layout split && s20 auto_again
