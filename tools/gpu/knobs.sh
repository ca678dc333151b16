# Schedule knobs on the smaller configs: concurrent vs phased class schedule, epilogue variant 3.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/knobs; mkdir -p $O
export TMPDIR=/tmp
b() { timeout -k 10 200 python -u bench.py --no-cpu-baseline "${@:2}" > $O/$1.log 2>&1; }
b s20 --scale 20 --steps 100 --warmup 10 && PR_HOT_PHASED=0 b s20_conc --scale 20 --steps 100 --warmup 10 && \
PR_CLASSES=16 PR_HOT_PHASED=0 b s20_c16conc --scale 20 --steps 100 --warmup 10 && \
b lj --graph lj --steps 50 --warmup 5 && PR_HOT_PHASED=0 b lj_conc --graph lj --steps 50 --warmup 5 && \
PR_EPI_VAR=3 b lj_v3 --graph lj --steps 50 --warmup 5 && \
b er --graph er --scale 24 --steps 20 --warmup 3 && PR_HOT_PHASED=0 b er_conc --graph er --scale 24 --steps 20 --warmup 3 && \
PR_EPI_VAR=3 b er_v3 --graph er --scale 24 --steps 20 --warmup 3
