# Layout / class-count A/B for the uniform (ER s24) and LiveJournal-shaped configs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/er_ab; mkdir -p $O
export TMPDIR=/tmp
er() { timeout -k 10 200 python -u bench.py --graph er --scale 24 --steps 20 --warmup 3 --no-cpu-baseline "${@:2}" > $O/er_$1.log 2>&1; }
lj() { timeout -k 10 150 python -u bench.py --graph lj --steps 50 --warmup 5 --no-cpu-baseline "${@:2}" > $O/lj_$1.log 2>&1; }
er auto && er fused --layout fused && PR_CLASSES=8 er c8 && PR_CLASSES=16 er c16 && PR_CLASSES=64 er c64 && \
lj fused --layout fused && PR_CLASSES=8 lj c8 && PR_CLASSES=32 lj c32 && lj auto
