# k_spmv_hot occupancy A/B at 64 classes, s26: one workgroup per CU with the full 16 K-slot hot set
# vs two co-resident workgroups per CU with a ~6 K-slot hot set each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/hotwg; mkdir -p $O
export TMPDIR=/tmp
run() { timeout -k 10 150 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/$1.log 2>&1; }
run base && PR_HOT_SLOTS=5900 run s5900_w1 && PR_HOT_SLOTS=5900 PR_HOT_WGS_PER_CU=2 run s5900_w2 && \
PR_HOT_SLOTS=16382 PR_HOT_WGS_PER_CU=2 run s16382_w2 && run base_again
